// Internal plan representation shared by the host plan compiler
// (plan.cpp) and the kernels/launchers (xdrgpu.hip).
#pragma once
#include <atomic>
#include <cstdint>
#include <mutex>
#include <vector>

#include "spec.h"
#include "xdrgpu.h"

namespace xdrg {

// One output word of a fixed-size program.  An output word is the OR of
// one or more terms; each term reads an 8-byte window of the input record
// (two consecutive 4-byte words starting at word `src`) and picks bytes
// with a v_perm_b32 selector (byte values 0-7 pick window bytes, 0x0C
// yields zero).  BOOL terms implement xdr_traits<bool> (types.h:335-349):
//   encode: wire = (native byte `sel` of word `src` != 0) as big-endian 1
//   decode: native byte `sel` = (wire word `src` != 0)
enum term_kind : uint16_t { T_PERM = 1, T_BOOL = 2 };
struct term {
  uint16_t kind;
  uint16_t src;  // input word index within the record
  uint32_t sel;  // v_perm selector (PERM) or byte position (BOOL)
};
// Index of the terms producing output word j: terms[start, start+count).
struct term_idx {
  uint16_t start;
  uint16_t count;
};
// Decode-time validation of one wire word (fixed plans).
enum check_kind : uint16_t { C_PAD = 1, C_ENUM = 2 };
struct check {
  uint16_t kind;
  uint16_t word;  // wire word index within the record
  uint32_t op;    // plan op index (error ordering)
  uint32_t a;     // PAD: register-order mask of bytes that must be zero; ENUM: table idx
  uint32_t b;     // ENUM: count
};

// Register-path program for one 16-byte chunk position: output word i of
// the chunk takes window pair (i & 2) of the same input chunk.
// Decode-side checks ride along (ck_kind 0 = none) so a lane holds its
// chunk's whole program in registers.
struct reg_word {
  uint32_t sel;
  uint32_t kind;     // T_PERM or T_BOOL (BOOL: sel = byte position)
  uint32_t ck_kind;  // 0, C_PAD or C_ENUM (decode only)
  uint32_t ck_op;
  uint32_t ck_a;
  uint32_t ck_b;
};

// Group-path program (non-identity fixed layouts, e.g. numerics): G records
// form a group whose input and output are whole 16-byte chunks; a lane owns
// one output chunk position q of every group it visits, and each of its 4
// output words is the OR of KT terms, each an 8-byte window at byte `off`
// of the group's input (4-byte aligned) picked with a v_perm selector, or a
// bool term (sel bit 31 set; low bits as term::sel of T_BOOL).  Unused
// terms select zero (sel 0x0C0C0C0C).
struct grp_term {
  uint32_t off;
  uint32_t sel;
};
constexpr uint32_t kGrpBool = 0x80000000u;
constexpr uint32_t kGrpHi = 0x40000000u;  // bool term reads the window's high word

struct fixed_prog {
  uint32_t in_words;   // words per input record
  uint32_t out_words;  // words per output record
  std::vector<term_idx> idx;  // [out_words]
  std::vector<term> terms;
  bool reg_ok = false;         // eligible for the register path
  std::vector<reg_word> reg;   // [out_words] when reg_ok
  uint32_t grp_G = 0;          // group path: records per group (0 = not eligible)
  uint32_t grp_C = 0;          //   output chunks per group
  uint32_t grp_KT = 0;         //   terms per output word
  std::vector<grp_term> grp;   //   [grp_C][4][grp_KT]
  bool has_bool = false;
};

// A plan's tables in one device's memory.
struct dev_tables {
  void *d_mem = nullptr;
  const xdrg_op *d_ops = nullptr;
  const uint32_t *d_table = nullptr;
  const term_idx *d_enc_idx = nullptr, *d_dec_idx = nullptr;
  const term *d_enc_terms = nullptr, *d_dec_terms = nullptr;
  const reg_word *d_enc_reg = nullptr, *d_dec_reg = nullptr;
  const grp_term *d_enc_grp = nullptr, *d_dec_grp = nullptr;
  const check *d_checks = nullptr;
};
constexpr int kMaxDevices = 64;

// Launch options of one plan (enum xdrg_plan_option); 0 / -1 = automatic.
struct plan_opts {
  int enc_kernel = 0;      // var encode: 0 auto, 1 per-lane, 3 chunk-map image
  int dec_kernel = 0;      // var decode: 0 auto, 1 per-lane, 2 window
  int fixed_path = 0;      // non-identity fixed plans: 0 auto (k_fixed_tile), 2 k_fixed_lds, 3 k_fixed_grp
  int image_bytes = -1;    // var encode LDS image per wave (-1: per plan)
  int window_bytes = -1;   // var decode LDS window per wave (-1: per call)
  int enc_unroll = 8;      // payload chunks in flight per lane (4, 8, 16)
  int dec_readahead = 1;   // window decode: 32-byte read-ahead past the window
  int size_linear = -1;    // size pass without a walk for linear plans: -1 when they have no generated
                           // size walk (its register-loaded records measured faster), 1 always, 0 never
  int grp_unroll = 0;      // group kernel: chunks in flight (0: per plan)
  int grp_blocks = 0;      // group kernel: workgroups (0: 2048)
  int grp_nontemporal = 0; // group kernel: non-temporal stores
  int specialize = 1;      // var plans: plan-specialized kernels (spec.cpp) when built
  int index_fast = 1;      // record index: speculative chain walk before the list ranking
                           // (1: the host waits for its flag; 2: asynchronous; 0: off)
  int stage_bytes = -1;    // window decode of packed plans: LDS stage of a group's arrays
  int enc_stream = -1;     // word-list plans: -1 walk-first record kernel, 1 + look-back (no size pass), 0 per-window walk
  int fixed_stream = -1;   // k_fixed_reg shape: -1 by working set, 0 plain/1024, 1 nt/one-shot, 2 plain/one-shot,
                           // 3 nt/1024
};

}  // namespace xdrg

struct xdrg_plan {
  std::vector<xdrg_op> ops;
  std::vector<uint32_t> table;
  uint32_t stride = 0;
  uint32_t fixed_size = 0;  // 0 => variable
  uint32_t path = 0;
  uint32_t max_depth = 0;
  uint32_t max_var_slots = 0;  // var plans: most opaque<>/string<> fields on one path
  uint32_t max_scalar_words = 0;  // var plans: most non-payload wire words on one path
  uint32_t max_pieces = 0;  // var plans: most 256-byte payload pieces on one path (by bounds)
  uint64_t max_record_bytes = 0;  // var plans: largest wire record the bounds allow
  uint64_t min_record_bytes = 0;  // smallest wire record (the record index needs >= 4)
  uint64_t max_chunks16 = 0;      // var plans: most 16-byte payload chunks on one path
  uint32_t max_slot_len = 0;      // var plans: largest opaque<>/string<> bound
  bool has_vector = false;        // xvector<T>/pointer<T> fields (XDRG_OP_VECTOR)
  bool has_sub = false;           // element subroutines (XDRG_F_SUB): the frame-walk kernels
  bool packed = false;            // decoded element arrays packed per 64-record group (no F_SUB)
  bool deep = false;              // subroutines can nest past XDRG_SUB_FRAMES (recursive types):
                                  // the frame walks add their deep passes (sub_kernels.h)
  uint32_t heap_factor = 0;       // decode element-area factor (xdrg_decode_heap_size)
  bool has_checks = false;
  bool has_bool = false;
  // var plans whose walk never branches (scalars, opaque[n], opaque<>,
  // string<>; no unions or containers): xdr_size = lin_base + the padded
  // lengths of the lin_n bytes fields whose xdrg_bytes_ref sit at lin_off[]
  bool linear = false;
  uint32_t lin_base = 0, lin_n = 0;
  uint32_t lin_off[8] = {};
  // fixed plans
  std::vector<uint32_t> op_wire_off;  // wire byte offset of each op (fixed)
  xdrg::fixed_prog enc, dec;
  std::vector<xdrg::check> checks;
  // Per-plan launch options (xdrg_plan_set_option): kernel choices and
  // launch shapes.  Set before the plan is shared between threads.
  xdrg::plan_opts opts;
  // Device copies of the tables, one allocation per device, made by the
  // plan's first launch on that device (plan creation never touches a
  // device).  Indexed by the HIP device ordinal current at the launch.
  std::mutex upload_mu;
  std::atomic<bool> uploaded[xdrg::kMaxDevices] = {};
  xdrg::dev_tables dev[xdrg::kMaxDevices];
  // plan-specialized kernels (var plans): generated source, code object,
  // per-device modules
  xdrg::spec_state spec;
};

namespace xdrg {
// Shared by the kernels' translation units (xdrgpu.hip, rpc.hip):
// exclusive scan of nb u64 block sums (in -> out; in != out lets it run on
// several workgroups), writing the total to
// status->total_bytes and offsets[n] (one workgroup, stream-ordered), and
// the thread's last-HIP-error record behind xdrg_last_hip_error.
int launch_block_scan(const unsigned long long *in, unsigned long long *out, uint32_t nb,
                      xdrg_status *status, uint64_t *offsets, uint64_t n, void *stream);
int record_hip_error(int hip_error, const char *what);
// Device fills and copies as kernels of the library's own (never memset or
// memcpy nodes in a captured graph: those do not take effect on replays
// after the first under ROCm's graph packet capture, profiles/r05e):
// `words` u32 of `value` at p (4-byte aligned), and n bytes src -> dst.
// Return a hipError_t.
int fill32(void *p, uint32_t value, uint64_t words, void *stream);
int copy_bytes(void *dst, const void *src, uint64_t n, void *stream);

// Validates ops and builds all host-side programs.  Returns XDRG_OK or an
// API error.  Does not touch the device.
int compile_plan(xdrg_plan &p);
}  // namespace xdrg
