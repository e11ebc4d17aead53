// Element subroutines (XDRG_F_SUB, include/xdrgpu.h): containers of
// variable-size elements and recursive types.
//
// xvector<T>/pointer<T> of a T that is not fixed-size (types.h:374-392,
// :476-512, :591-665) archives each element with xdr_traits<T>::save/load,
// which for a struct or union walks its fields (xdrc/gen_hh.cc:212-250,
// :575-675) -- and T may contain the container again (test_recursive,
// tests/xdrtest.x:29-33; rpcbind's rp__list, xdrpp/rpcb_prot.x:34).  The
// plan gives such an element a subroutine: ops after the record's END,
// entered once per element.  These kernels walk one record per lane with an
// explicit stack of element frames (the reference recurses on the C++
// stack; marshal.h:129-136, :198-205 count its levels):
//
//   k_sub_size     xdr_size per record (+ depth_checker levels) and the
//                  64-record block sums;
//   k_sub_encode   xdr_generic_put of the record (marshal.h:84-137);
//   k_sub_decode   xdr_generic_get (marshal.h:142-211); decoded element
//                  arrays are carved from the record's element area.
//
// Nesting is bounded only by the data (and marshaling_stack_limit).  Each
// kernel runs as up to three passes over the same walk:
//   main   one lane per record, kSubFrames frames in registers (a push or
//          pop shifts them, so every index is a constant and the kernel uses
//          no scratch); a record that needs more is appended to list A and
//          left alone;
//   deep A a fixed grid of kDeepLanesA lanes walks list A, kDeepSlabA frames
//          per lane in the frame pool (global memory); a record that needs
//          more goes to list B;
//   deep B kDeepLanesB lanes walk list B with kDeepSlabB frames each; a
//          record that needs more is xdr_stack_overflow at the VECTOR op
//          that would open the frame (the reference's own recursion ends in
//          a segmentation fault far earlier: xdr_from_opaque of a
//          test_recursive chain between 60K and 100K levels, xdr_to_opaque
//          between 100K and 200K, g++ -O2 on an 8 MiB stack).
// The encode pass reuses the lists its size pass built (the two walks visit
// the same frames), so it defers nothing itself.  A deferred record is
// walked again from its start by the next pass: every write it makes is
// deterministic, so the main pass's partial output is simply overwritten.
//
// A body's field offsets are element-relative and its depths relative to
// the VECTOR op that entered it.  Fixed-size element containers inside a
// body keep the inline element walk of xdrgpu.hip.
//
// Included by xdrgpu.hip after its element helpers (load_ops, union_target,
// enc_vector_elems, dec_vector_elems).
//
// Each walk visits one op per step through an op policy OPS::visit(ops, pc,
// step): rt_ops hands it the plan op from LDS (the library's kernels,
// xdrgpu.hip); a generated module's plan_ops (codegen.cpp, recursive plans)
// switches on pc to the op as compile-time constants, and lets a scalar op
// fall through to the next one, so a straight run of fields is one step.
#pragma once
#include "elem_kernels.h"

namespace xdrg {
namespace dev {

constexpr uint32_t kSubFrames = XDRG_SUB_FRAMES;  // register frames of the main pass
constexpr uint32_t kReported = 0x100;  // decode: the element walk reported the error

// One open container: its current element (heap byte offset), the elements
// after it, the VECTOR op (stride and body pc come from the op) and where
// the walk goes on when the container closes (vd: op in the low 16 bits,
// return pc in the high 16; plans have fewer than kOpRecordLevel ops), and
// the levels its pop gives back (the op's depth, plus those of the frames
// it replaced -- sub_tail), and the frames it stands for (1 + those).
struct sub_frame {
  uint64_t eb;
  uint32_t left;
  uint32_t vd;
  uint32_t dsum;
  uint32_t nf;
  __device__ __forceinline__ uint32_t vpc() const { return vd & 0xffffu; }
  __device__ __forceinline__ uint32_t ret() const { return vd >> 16; }
};
__device__ __forceinline__ sub_frame make_frame(uint64_t eb, uint32_t left, uint32_t vpc, uint32_t ret,
                                                uint32_t dsum, uint32_t nf) {
  return sub_frame{eb, left, vpc | (ret << 16), dsum, nf};
}

// The walks touch the top frame only (and, after an error in the decode,
// every open frame once): top / push / pop / each with fp = the frames open.
//
// Main pass: the frames in registers, f[0] the top one, pushed and popped by
// shifting (every index is a constant once unrolled), so the kernels use no
// private (scratch) memory.  A hipGraph replayed more than once faulted
// with HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in the frame walks while
// their frames lived in private memory (520 B of scratch a lane): the
// second and later replays under ROCm's graph packet capture
// (DEBUG_CLR_GRAPH_PACKET_CAPTURE, on by default); the same graph replayed
// 4 times bit-exact with the packet capture off, and graphs of
// scratch-free kernels replay under it (profiles/r05a, r05b).
template <uint32_t K>
struct reg_stack_t {
  sub_frame f[K];
  __device__ __forceinline__ sub_frame &top(uint32_t) { return f[0]; }
  __device__ __forceinline__ void push(uint32_t, const sub_frame &x) {
#pragma unroll
    for (int j = K - 1; j > 0; --j) f[j] = f[j - 1];
    f[0] = x;
  }
  __device__ __forceinline__ void pop(uint32_t) {
#pragma unroll
    for (int j = 0; j + 1 < static_cast<int>(K); ++j) f[j] = f[j + 1];
  }
  // fn(k, frame k, frame k - 1) for each of the fp open frames (k = 0 is
  // the bottom one; its "frame below" is unused)
  template <class FN> __device__ __forceinline__ void each(uint32_t fp, FN &&fn) const {
#pragma unroll
    for (uint32_t j = 0; j < K; ++j)
      if (j < fp) fn(fp - 1u - j, f[j], f[j + 1 < K ? j + 1 : j]);
  }
  __device__ __forceinline__ uint32_t cap() const { return K; }
  static constexpr bool kRegs = true;
  static constexpr uint32_t kCap = K;
  uint32_t lf = 0;  // the frames open, replaced ones included (sub_open)
};
using reg_stack = reg_stack_t<kSubFrames>;
// The decode's wave pass ("Long records"): its frames are scalar registers,
// fewer of them (a list takes one; a record that needs more goes to deep
// pass A).  Eight spilled 117 SGPRs, four 30: rp_list's wave pass 0.89 ->
// 0.81 ms (profiles/r05w7).
constexpr uint32_t kWaveFrames = 4;
using wave_stack = reg_stack_t<kWaveFrames>;
static_assert(kWaveFrames != kSubFrames, "the decode tells its passes apart by their stacks' frames");
// Deep passes: `n` frames per lane in the caller's workspace.
struct slab_stack {
  sub_frame *f;
  uint32_t n;
  __device__ __forceinline__ sub_frame &top(uint32_t fp) { return f[fp - 1]; }
  __device__ __forceinline__ void push(uint32_t fp, const sub_frame &x) { f[fp] = x; }
  __device__ __forceinline__ void pop(uint32_t) {}
  template <class FN> __device__ __forceinline__ void each(uint32_t fp, FN &&fn) const {
    for (uint32_t k = 0; k < fp; ++k) fn(k, f[k], f[k ? k - 1 : 0]);
  }
  __device__ __forceinline__ uint32_t cap() const { return n; }
  static constexpr bool kRegs = false;
  static constexpr uint32_t kCap = 0;
  uint32_t lf = 0;
};

// Tail containers.  A container of element subroutines whose elements are
// the last thing the element enclosing it does (the op after it, through
// jumps, is its body's END), opened while that element is its container's
// last one: when it closes, so does the frame below.  Its frame replaces
// that one instead of going on top, and takes over its return pc -- a
// linked list (rp__list's rpcb_next, xdrpp/rpcb_prot.x:34; test_recursive's
// nextvec, tests/xdrtest.x:29-33) walks in one frame however long it is,
// in the main pass.  The depth levels of the replaced frames stay counted
// (dsum) and are given back at the pop; so do the frames themselves (nf):
// XDRG_MAX_FRAMES open frames, replaced ones included, is xdr_stack_overflow
// in any pass (as running out of the last pass's frames is), which also
// ends a walk around a cycle in a staged heap.
__device__ __forceinline__ bool sub_tail(const xdrg_op *__restrict__ ops, uint32_t pc) {
  uint32_t q = pc + 1;
  while (ops[q].kind == XDRG_OP_JUMP) q = ops[q].arg0;
  return ops[q].kind == XDRG_OP_END;
}
// Open the container at pc (count cnt >= 1, first element eb): on top of
// the stack, or in place of the top frame (sub_tail; allow_tail).  Returns
// kOpenOk (*tail set when it replaced a frame), kOpenFull when the stack is
// full (the next pass takes the record), or kOpenOver at XDRG_MAX_FRAMES.
enum : int { kOpenOk = 0, kOpenFull = 1, kOpenOver = 2 };
template <class ST>
__device__ __forceinline__ int sub_open(const xdrg_op *__restrict__ ops, ST &st, uint32_t &fp, uint32_t pc,
                                        uint32_t depth, uint64_t eb, uint32_t cnt, bool allow_tail, bool *tail) {
  if (st.lf >= XDRG_MAX_FRAMES) return kOpenOver;
  if (allow_tail && fp && st.top(fp).left == 0u && sub_tail(ops, pc)) {
    sub_frame &t = st.top(fp);
    t = make_frame(eb, cnt - 1u, pc, t.ret(), t.dsum + depth, t.nf + 1u);
    ++st.lf;
    *tail = true;
    return kOpenOk;
  }
  if (fp == st.cap()) return kOpenFull;
  st.push(fp++, make_frame(eb, cnt - 1u, pc, pc + 1u, depth, 1u));
  ++st.lf;
  return kOpenOk;
}

// The pass a launch runs (see the top of the file).
struct sub_pass {
  const uint32_t *list;            // deep: the records to walk (nullptr: main pass, every record)
  const unsigned long long *count; //       and their number
  uint32_t *defer;                 // where records that need more frames go (nullptr: see last)
  unsigned long long *defer_count;
  sub_frame *slabs;                // deep: `slab` frames per lane
  uint32_t slab;
  uint32_t last;                   // 1: running out of frames is xdr_stack_overflow
  uint32_t packed;                 // decode, main pass of a non-recursive plan: packed element areas
  uint32_t lines;                  // encode, main pass: the host gave each lane a 64-byte line buffer
  // The chain log (recursive plans' size and encode main passes; see
  // "Chains" below): null when the host gave none.
  uint32_t *chain_of;              // per record: the chain its size walk logged, or ~0
  uint32_t *chain_rec;             // per chain: its record
  uint32_t *chain_end;             // per chain: the record's bytes where the chain closes
  struct sub_node *nodes;          // the logged nodes
  unsigned long long *chain_cnt;   // allocation counters (zeroed per call)
  unsigned long long *node_cnt;
  uint32_t chain_cap, node_cap;
  // The decode's wave pass (see "Long records" below): the main pass lists
  // records of kWaveMin bytes or more here (null: it walks them itself);
  // wave = 1: this launch is the wave pass (list / count are that list).
  uint32_t *wave_list;
  unsigned long long *wave_count;
  uint32_t wave;
  // decode, main pass: the host gave each wave kWaveBlk bytes of LDS after
  // the ops, for the stream of its 64 records (win_rd); wave pass: each
  // wave also has kWaveBlk / 2 bytes after the blocks for list_decode's
  // node candidates
  uint32_t win;
  // size, main pass: per chain, where the chain pass takes it over (see
  // "Chains"; null: the size walk chases every chain itself)
  struct sub_node *heads;
};

// Long records (decode).  A lane's walk of its record reads the stream a
// word at a time, and on CDNA one counter covers a wave's loads and stores:
// each read waits for every store the walk issued before it, a memory round
// trip a field -- a 500-node rp__list took one lane 2.6 ms (profiles/r05end2).
// The main pass lists records of kWaveMin bytes or more instead, and the
// wave pass walks each with a whole wave in step (the same values in every
// lane) from a block of the record in LDS (wave_rd): a read waits only on
// LDS, and a block reload -- kWaveBlk bytes, 16 bytes a lane per load -- is
// the one round trip per block.  Each word read goes to a scalar register
// (readfirstlane), so the walk's values, branches and addresses are scalar
// work.  Its frames are the main pass's (registers, tail containers); a
// record they cannot finish goes to deep pass A as from the main pass.
// rp_list (profiles/r05w2-w4): decode 2.60 -> 1.66 ms (main pass 0.46 ms,
// wave pass 1.14 ms with vector values); the last 16 bytes read kept in
// registers (a run of fields one LDS read per four words) was slower, 1.22
// ms.  Walking the long records inside the main pass instead
// (each wave its own, after its lanes' walks) was slower, 2.16 ms (1.83 with
// the register line): the walks share their SIMDs with the pass's waves, and
// two walk instances in one kernel spilled (288 bytes of scratch).
constexpr uint32_t kWaveMin = 4096;
constexpr uint32_t kWaveBlk = 8192;  // bytes of LDS per wave
constexpr uint32_t kWaveWaves = 4;   // waves per workgroup of the wave pass

template <class T> struct no_ref_t { using type = T; };
template <class T> struct no_ref_t<T &> { using type = T; };
template <class T> using no_ref = typename no_ref_t<T>::type;  // (runtime-compiled modules have no <type_traits>)

// The stream as a walk reads it: a lane's own global loads ...
struct glob_rd {
  const uint8_t *xdr;
  static constexpr bool kWave = false;
  __device__ __forceinline__ uint32_t operator()(uint64_t q) const { return ld32(xdr + q); }
};
// ... or, in the decode's main pass, the wave's window: the stream of its
// 64 records (their first kWaveBlk bytes) loaded to LDS by the whole wave
// before the walks, so a lane's read of its record waits on LDS, not on the
// stores its walk issued before (lim = 0: no window, every read global) ...
struct win_rd {
  const uint8_t *xdr;
  const uint32_t *buf;
  uint64_t base;  // stream offset of buf[0]
  uint32_t lim;   // bytes of the window
  static constexpr bool kWave = false;
  __device__ __forceinline__ uint32_t operator()(uint64_t q) const {
    const uint64_t d = q - base;
    return d < lim ? buf[d >> 2] : ld32(xdr + q);
  }
};
// ... or the wave pass's LDS block of the record [.., end) (end and every
// position read a multiple of 4; positions below end only).
struct wave_rd {
  const uint8_t *xdr;
  uint64_t end;
  uint32_t *buf;          // kWaveBlk bytes of LDS
  mutable uint64_t base;  // stream offset of buf[0] (16-byte aligned; ~0: none)
  static constexpr bool kWave = true;
  __device__ __forceinline__ uint32_t operator()(uint64_t q) const {
    if (q < base || q - base >= kWaveBlk) {
      const uint64_t b0 = q & ~15ull;
      wave_sync();  // every lane past its reads of the old block
#pragma unroll
      for (uint32_t j = 0; j < kWaveBlk / 1024u; ++j) {
        const uint32_t k = (threadIdx.x & 63u) + 64u * j;
        const uint64_t o = b0 + 16ull * k;
        u32x4 v{0u, 0u, 0u, 0u};
        if (o + 16 <= end) {
          v = ld16u(xdr + o);
        } else if (o < end) {
          v.x = ld32(xdr + o);
          if (o + 8 <= end) v.y = ld32(xdr + o + 4);
          if (o + 12 <= end) v.z = ld32(xdr + o + 8);
        }
        *reinterpret_cast<u32x4 *>(buf + 4u * k) = v;
      }
      wave_sync();
      base = b0;
    }
    // the same word in every lane: scalar from here on (the walk's values,
    // branches and addresses become SGPR work)
    return __builtin_amdgcn_readfirstlane(buf[(q - base) >> 2]);
  }
};
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v))) |
         (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32))) << 32);
}
// Zero `bytes` (a multiple of 4) at p: the wave pass spreads the stores over
// its lanes (one store instruction per 256 bytes, not per word).
template <class RD>
__device__ __forceinline__ void zero_words(uint8_t *p, uint64_t bytes) {
  if constexpr (RD::kWave) {
    for (uint64_t z = 4u * (threadIdx.x & 63u); z < bytes; z += 256u) st32(p + z, 0u);
  } else {
    for (uint64_t z = 0; z < bytes; z += 4) st32(p + z, 0u);
  }
}

// Chains.  A linked list walks in one frame (sub_tail), but one lane still
// walks it node after node: a 500-node rp__list made the main passes one
// lane's walk long (the encode 3.1 ms for 1M lists, its pointer chase ~2
// us a node under the load of the million short ones).  The size pass
// chases it anyway, so it logs the chain: at the kChainT-th frame
// replacement of the first chain of a record to get that far (each
// replacement opening a one-element container), every node from there to
// the chain's end -- its element, its first byte in the record's stream
// and its depth base -- and the record's byte count where the chain closes.
// The encode's main pass then writes the record up to that node, jumps to
// where the chain closes and goes on from there, and a node pass
// (sub_chain_kernel) writes the logged nodes, one lane each: the chain in
// parallel.  A chain that opens a container of more than one element, a
// record the main pass does not finish, or a full log leaves the record
// unlogged (chain_of ~0): its walk writes it all, as before.
// The size walk's own chase of a long chain was then its critical path (one
// lane, a round trip a node: 1.3 ms for rp_list's 500-node lists), so a
// chain whose close ends the record -- an optional (`*`, at most one
// element) tail container in the record's only frame, rp__list's rpcb_next
// -- is handed over at that node instead (heads[c]: the node, its first
// byte, depth base and the frames open), and the chain pass
// (sub_chain_size_kernel) sizes it a wave at a time: each lane loads the
// node a stride further on (the element size, then the spacing seen), sizes
// it to its chain's count word and reads its link; the nodes from the
// wave's first on whose links each lead to the next lane's are the chain's
// (every address is checked against its predecessor's link, so a heap laid
// out otherwise costs a round trip a node, as the lane's chase did), their
// first bytes a prefix sum, and they are logged as the lane would have.
constexpr uint32_t kChainT = 32;
struct sub_node {
  uint64_t eb;     // the node's element (heap offset)
  uint32_t s;      // its first byte, record-relative (after its count word)
  uint32_t dbase;  // the depth levels open at its first field
  uint32_t chain;  // its chain (~0: an unused slot)
  uint32_t vpc;    // the chain's VECTOR op (the node ends with its count word)
};
constexpr uint32_t kChainChunk = 64;  // nodes a lane claims at a time

enum : int { kWalkCont = -1, kWalkOk = 0, kWalkErr = 1, kWalkFull = 2, kWalkChain = 3 };

// The interpreted op policy: the op from the plan table (LDS).
struct rt_ops {
  static constexpr uint32_t kImgWords = 0;  // field offsets at run time: no element image
  template <class F>
  __device__ __forceinline__ static int visit(const xdrg_op *__restrict__ ops, uint32_t &pc, F &&step) {
    return step(ops[pc]);
  }
};

// A plan op as compile-time constants (generated op policies).
template <uint32_t K, uint32_t F, uint32_t D, uint32_t NOFF, uint32_t A0, uint32_t A1, uint32_t A2, uint32_t A3,
          uint32_t A4>
struct xop {
  static constexpr uint8_t kind = K;
  static constexpr uint8_t flags = F;
  static constexpr uint16_t depth = D;
  static constexpr uint32_t noff = NOFF, arg0 = A0, arg1 = A1, arg2 = A2, arg3 = A3, arg4 = A4;
};

// A running out of frames: defer the record to the next pass, or report.
__device__ __forceinline__ void sub_full(const sub_pass &P, uint64_t r, uint32_t pc, uint32_t code,
                                         unsigned long long *err) {
  if (P.defer) P.defer[atomicAdd(P.defer_count, 1ull)] = static_cast<uint32_t>(r);
  else if (P.last) report(err, r, pc, code);
}

// The native object a lane's walk is in: its record (frame 0, `len` bytes)
// or an element in the heap.  Heap bytes at or past heap_len read as 0.
// IW > 0 (generated walks, whose field offsets are constants): the current
// element's first 4*IW bytes in registers, loaded whole each time the walk
// enters an element (refresh) -- one round trip per element where the
// field-by-field reads made one per field along rp__list's chain.
template <uint32_t IW>
struct sub_src_t {
  const uint8_t *nat;
  uint32_t len;
  const uint8_t *heap;
  uint64_t heap_len;
  uint64_t eb;
  bool in_heap;
  uint32_t img[IW ? IW : 1];
  __device__ __forceinline__ void refresh() {
    if constexpr (IW > 0) {
      if (!in_heap) return;
      if (!(eb & 3u) && eb + 4u * IW <= heap_len) {
#pragma unroll
        for (uint32_t q = 0; q + 4 <= IW; q += 4) {
          const u32x4 t = ld16u(heap + eb + 4u * q);
          img[q] = t.x;
          img[q + 1] = t.y;
          img[q + 2] = t.z;
          img[q + 3] = t.w;
        }
#pragma unroll
        for (uint32_t q = IW & ~3u; q < IW; ++q) img[q] = ld32(heap + eb + 4u * q);
      } else {
#pragma unroll
        for (uint32_t q = 0; q < IW; ++q) img[q] = hword(eb + 4u * q);
      }
    }
  }
  __device__ __forceinline__ bool cached(uint32_t off) const { return IW > 0 && in_heap && off / 4u < IW; }
  // a heap word at any byte offset
  __device__ __forceinline__ uint32_t hword(uint64_t off) const { return unaligned_word(heap, heap_len, off); }
  // the four heap words at any byte offset, their loads issued together
  __device__ __forceinline__ void hwords4(uint64_t off, uint32_t (&w)[4]) const {
    const uint64_t a = off & ~3ull;
    const uint32_t sh = static_cast<uint32_t>(off & 3u);
    if (a + 20 <= heap_len) {
      const u32x4 t = ld16u(heap + a);
      const uint32_t t4 = sh ? ld32(heap + a + 16) : 0u;
      w[0] = __builtin_amdgcn_alignbyte(t.y, t.x, sh);
      w[1] = __builtin_amdgcn_alignbyte(t.z, t.y, sh);
      w[2] = __builtin_amdgcn_alignbyte(t.w, t.z, sh);
      w[3] = __builtin_amdgcn_alignbyte(t4, t.w, sh);
    } else {
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) w[j] = hword(off + 4u * j);
    }
  }
  // a naturally aligned field word
  __device__ __forceinline__ uint32_t w(uint32_t off) const {
    if (cached(off)) return img[off / 4u];
    return in_heap ? hword(eb + off) : ld32(nat + off);
  }
  // a word at any byte offset (opaque[n] fields)
  __device__ __forceinline__ uint32_t wu(uint32_t off) const {
    if (!(off & 3u) && cached(off)) return img[off / 4u];
    return in_heap ? hword(eb + off) : unaligned_word(nat, len, off);
  }
  __device__ __forceinline__ uint32_t b(uint32_t off) const {
    if (cached(off)) return (img[off / 4u] >> (8u * (off & 3u))) & 0xffu;
    return in_heap ? (hword(eb + off) & 0xffu) : nat[off];
  }
  __device__ __forceinline__ uint64_t w64(uint32_t off) const {
    return static_cast<uint64_t>(w(off)) | (static_cast<uint64_t>(w(off + 4)) << 32);
  }
};

// Pop finished elements: returns false when the record's own END is
// reached, else sets pc (and the walk's object and depth) to the next
// element's body or the op after the container.
template <class ST>
__device__ __forceinline__ bool sub_next(const xdrg_op *__restrict__ ops, ST &st, uint32_t &fp, uint32_t &pc,
                                         uint32_t &dbase, uint64_t &eb, bool &in_heap) {
  if (!fp) return false;
  sub_frame &f = st.top(fp);
  const xdrg_op &v = ops[f.vpc()];
  if (f.left) {
    --f.left;
    f.eb += v.arg1;
    eb = f.eb;
    pc = v.arg4;
    return true;
  }
  pc = f.ret();
  dbase -= f.dsum;
  st.lf -= f.nf;
  st.pop(fp);
  if (--fp) eb = st.top(fp).eb;
  else in_heap = false;
  return true;
}

// The walk of one record for a pass: the main pass walks record gid, a
// deep pass every listed record its lane owns.
template <bool WAVE = false, class F>
__device__ __forceinline__ void sub_records(const sub_pass &P, uint64_t n, F &&walk) {
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (!P.list) {
    if (gid < n) {
      reg_stack st;
      walk(gid, st);
    }
    return;
  }
  const uint64_t cnt = *P.count, lanes = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  if constexpr (WAVE) {
    if (P.wave) {  // a listed record per wave, every lane on its walk
      wave_stack st;
      for (uint64_t i = gid / 64u; i < cnt; i += lanes / 64u) walk(static_cast<uint64_t>(P.list[i]), st);
      return;
    }
  }
  slab_stack st{P.slabs + gid * P.slab, P.slab};
  for (uint64_t i = gid; i < cnt; i += lanes) walk(static_cast<uint64_t>(P.list[i]), st);
}

// The size walk's side of the chain log (see "Chains"): one per record.
struct chain_logger {
  sub_pass P;  // (a copy: the kernel argument's address would put it in private memory)
  bool on;     // false: no log (deep passes, or the host gave none)
  uint64_t r;
  uint32_t c = ~0u;     // the chain being logged
  uint32_t cfin = ~0u;  // the chain logged to its close
  uint32_t lfp = 0;     // its frame level
  uint32_t vpc0 = ~0u;  // the VECTOR op its replacements open
  bool done = false;    // the record's first chain past kChainT was met
  uint64_t at = 0, end = 0;  // this lane's claimed node slots
  __device__ __forceinline__ void start(uint32_t fp, uint32_t vpc) {
    const unsigned long long k = atomicAdd(P.chain_cnt, 1ull);
    if (k >= P.chain_cap) return;
    c = static_cast<uint32_t>(k);
    lfp = fp;
    vpc0 = vpc;
    P.chain_rec[c] = static_cast<uint32_t>(r);
    if (P.heads) P.heads[c].chain = ~0u;  // (not handed over, unless below)
  }
  // not a chain the node pass takes: the record's walks write it whole, and
  // the node pass skips the nodes logged so far
  __device__ __forceinline__ void drop() {
    P.chain_rec[c] = ~0u;
    c = ~0u;
  }
  __device__ __forceinline__ void add(uint64_t eb, uint64_t s, uint32_t dbase, uint32_t vpc) {
    if (at == end) {
      const unsigned long long a = atomicAdd(P.node_cnt, static_cast<unsigned long long>(kChainChunk));
      if (a + kChainChunk > P.node_cap) {  // the log is full: this record walks its chain itself
        c = ~0u;
        return;
      }
      at = a;
      end = a + kChainChunk;
    }
    P.nodes[at++] = sub_node{eb, static_cast<uint32_t>(s), dbase, c, vpc};
  }
  __device__ __forceinline__ void close(uint64_t s) {
    P.chain_end[c] = static_cast<uint32_t>(s);
    cfin = c;
    c = ~0u;
  }
  // the walk is over (ok: it sized the record): the record's chain, and the
  // claimed slots it did not fill marked unused
  __device__ __forceinline__ void finish(bool ok) {
    if (!on) return;
    for (; at < end; ++at) P.nodes[at].chain = ~0u;
    P.chain_of[r] = ok && c == ~0u ? cfin : ~0u;
  }
};

// ---------------------------------------------------------------- size
// xdr_size (xdr_traits<T>::serial_size) of one record, and with DEPTH the
// deepest class/container level its walk enters (depth_checker,
// xdrpp/depth_checker.h:41-54).  kWalkErr with the op and code: a bad
// discriminant or a record of 2^31 bytes or more; kWalkFull (op in bad_op):
// the stack ran out.
// NODE (the chain pass): one node of a chain from its element body (nd.pc)
// to its chain's count word (the VECTOR op nd.stop in the element's own
// frame), with nd.lf frames open (replaced ones included); nd.next / nd.cnt
// are that count word's container.
struct sub_size_node {
  uint32_t pc = 0, stop = ~0u, lf = 0, cnt = 0;
  uint64_t next = 0;
};
// A tail container's frame whose return is the record's END (the walk ends
// when the chain closes).
__device__ __forceinline__ bool sub_ret_end(const xdrg_op *__restrict__ ops, uint32_t q) {
  while (ops[q].kind == XDRG_OP_JUMP) q = ops[q].arg0;
  return ops[q].kind == XDRG_OP_END;
}
template <bool DEPTH, class OPS, class ST, bool NODE = false>
__device__ __forceinline__ int sub_size(const xdrg_op *__restrict__ ops, const uint32_t *__restrict__ table,
                        sub_src_t<OPS::kImgWords> src,
                        uint64_t &s, uint32_t &dmax, uint32_t &bad_op, uint32_t &code, ST &st, chain_logger &lg,
                        sub_size_node *nd = nullptr) {
  uint32_t fp = 0, pc = NODE ? nd->pc : 0, dbase = 0;
  st.lf = NODE ? nd->lf : 0;
  auto step = [&](const auto &op) __attribute__((always_inline)) -> int {
    if (op.kind == XDRG_OP_END) {
      // (the logged chain closes when its frame pops)
      const bool closing = lg.c != ~0u && fp == lg.lfp && st.top(fp).left == 0u;
      if (!sub_next(ops, st, fp, pc, dbase, src.eb, src.in_heap)) return kWalkOk;
      if (closing) lg.close(s);
      src.refresh();
      return kWalkCont;
    }
    if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; return kWalkCont; }
    if (DEPTH) dmax = max(dmax, dbase + op.depth);
    switch (op.kind) {
    case XDRG_OP_U64: s += 8; ++pc; break;
    case XDRG_OP_OPAQUE: s += (op.arg0 + 3u) & ~3u; ++pc; break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
      s += 4ull + ((static_cast<uint64_t>(src.w(op.noff + 8)) + 3u) & ~3ull);
      ++pc;
      break;
    case XDRG_OP_UNION: {
      const int t = union_target(op, table, src.w(op.noff));
      s += 4;
      if (t < 0) { bad_op = pc; code = XDRG_ERR_BAD_DISCRIMINANT; return kWalkErr; }
      pc = static_cast<uint32_t>(t);
      break;
    }
    case XDRG_OP_VECTOR: {
      const uint32_t cnt = src.w(op.noff + 8);
      s += 4;
      if (!(op.flags & XDRG_F_SUB)) {  // fixed-size elements (arg3 wire bytes each)
        s += static_cast<uint64_t>(cnt) * op.arg3;
        if (DEPTH && cnt)
          for (uint32_t k = 1; k <= op.arg2; ++k) dmax = max(dmax, dbase + ops[pc + k].depth);
        pc += 1 + op.arg2;
        break;
      }
      if (NODE && fp == 0 && pc == nd->stop) {  // the node's count word: its link
        nd->next = src.w64(op.noff);
        nd->cnt = cnt;
        if (cnt && st.lf >= XDRG_MAX_FRAMES) { bad_op = pc; code = XDRG_ERR_STACK_PUT; return kWalkErr; }
        return kWalkOk;
      }
      if (!cnt) { ++pc; break; }
      bool tail = false;
      const int o = sub_open(ops, st, fp, pc, op.depth, src.w64(op.noff), cnt, true, &tail);
      if (o == kOpenFull) { bad_op = pc; return kWalkFull; }
      if (o == kOpenOver) { bad_op = pc; code = XDRG_ERR_STACK_PUT; return kWalkErr; }
      dbase += op.depth;
      src.eb = st.top(fp).eb;
      src.in_heap = true;
      if (lg.on && tail) {  // a frame replaced: the chain log
        if (lg.c == ~0u) {
          if (!lg.done && st.top(fp).nf == kChainT + 1u) {  // the record's first chain this long
            lg.done = true;
            if (cnt == 1u) lg.start(fp, pc);
            // handed over to the chain pass: a chain whose close ends the record
            if (!DEPTH && lg.c != ~0u && lg.P.heads && fp == 1u && op.arg0 == 1u && sub_ret_end(ops, st.top(fp).ret())) {
              lg.P.heads[lg.c] = sub_node{src.eb, static_cast<uint32_t>(s), dbase, st.lf, pc};
              lg.cfin = lg.c;
              lg.c = ~0u;
              return kWalkChain;
            }
          }
        } else if (fp == lg.lfp && (cnt != 1u || pc != lg.vpc0)) {
          // more than one element, or a node of another type (a chain that
          // alternates tail containers: a node's walk in the node pass stops
          // at its own chain's count word only when every node opens the same)
          lg.drop();
        }
        if (lg.c != ~0u && fp == lg.lfp) lg.add(src.eb, s, dbase, pc);
      }
      src.refresh();
      pc = op.arg4;
      break;
    }
    default: s += 4; ++pc; break;
    }
    // every frame adds a count word, so a walk that never ends (a cycle in
    // the staged heap) fails here or at its last frame
    if (s >= kSizeErr) { bad_op = 0; code = XDRG_ERR_OVERFLOW_PUT; return kWalkErr; }
    return kWalkCont;
  };
  for (;;) {
    const int rc = OPS::visit(ops, pc, step);
    if (rc != kWalkCont) return rc;
  }
}

// Kernel parameters of the three walks: the library's kernels (xdrgpu.hip,
// rt_ops) and the generated ones (codegen.cpp, plan_ops) take the same.
#define XDRG_SUB_SIZE_PARAMS                                                                                      \
  const uint8_t *__restrict__ native, uint64_t n, uint32_t stride, const uint8_t *__restrict__ heap,               \
      uint64_t heap_len, const xdrg_op *__restrict__ ops, uint32_t nops, const uint32_t *__restrict__ table,       \
      uint32_t *__restrict__ sizes, unsigned long long *__restrict__ block_sums, uint32_t mark,                    \
      unsigned long long *err, uint32_t *__restrict__ depths, xdrg::dev::sub_pass P
#define XDRG_SUB_SIZE_ARGS native, n, stride, heap, heap_len, ops, nops, table, sizes, block_sums, mark, err, depths, P
#define XDRG_SUB_ENCODE_PARAMS                                                                                    \
  const uint8_t *__restrict__ native, uint64_t n, uint32_t stride, const uint8_t *__restrict__ heap,               \
      uint64_t heap_len, uint8_t *__restrict__ xdr, uint64_t cap, uint64_t *__restrict__ offsets,                  \
      const uint32_t *__restrict__ sizes, const unsigned long long *__restrict__ block_base,                       \
      const xdrg_op *__restrict__ ops, uint32_t nops, const uint32_t *__restrict__ table, uint32_t stack_limit,    \
      uint32_t mark, unsigned long long *err, xdrg::dev::sub_pass P
#define XDRG_SUB_ENCODE_ARGS                                                                                      \
  native, n, stride, heap, heap_len, xdr, cap, offsets, sizes, block_base, ops, nops, table, stack_limit, mark, err, P
#define XDRG_SUB_DECODE_PARAMS                                                                                    \
  const uint8_t *__restrict__ xdr, uint64_t len, const uint64_t *__restrict__ offsets, uint64_t n,                 \
      uint8_t *__restrict__ native, uint32_t stride, const xdrg_op *__restrict__ ops, uint32_t nops,               \
      const uint32_t *__restrict__ table, uint32_t stack_limit, uint8_t *__restrict__ heap, uint64_t ebase,        \
      uint32_t F, uint32_t mark, unsigned long long *err, xdrg::dev::sub_pass P
#define XDRG_SUB_DECODE_ARGS                                                                                      \
  xdr, len, offsets, n, native, stride, ops, nops, table, stack_limit, heap, ebase, F, mark, err, P

template <bool DEPTH, class OPS>
__device__ __forceinline__ void sub_size_kernel(XDRG_SUB_SIZE_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  load_ops(sops, ops, nops);
  uint32_t size = 0;  // main pass: this lane's contribution to its block sum
  sub_records(P, n, [&](uint64_t r, auto &st) {
    const sub_src_t<OPS::kImgWords> src{native + r * stride, stride, heap, heap_len, 0, false, {}};
    uint64_t s = mark;
    uint32_t dmax = 0, bad_op = 0, code = 0, sz = kSizeErr;
    chain_logger lg{P, !P.list && P.chain_of, r};
    const int rc = sub_size<DEPTH, OPS>(sops, table, src, s, dmax, bad_op, code, st, lg);
    lg.finish(rc == kWalkOk || rc == kWalkChain);
    if (rc == kWalkOk || rc == kWalkChain) {  // (a chain handed over: its bytes so far, the chain pass adds the rest)
      sz = static_cast<uint32_t>(s);
    } else if (rc == kWalkErr) {
      report(err, r, bad_op, code);
    } else {  // the stack ran out
      sub_full(P, r, bad_op, XDRG_ERR_STACK_PUT, err);
      if (!P.last) return;  // the next pass sizes it
    }
    if (sizes) sizes[r] = sz;
    if (DEPTH) depths[r] = dmax;
    if (!P.list) size = sz;
    else if (block_sums && !(sz & kSizeErr)) atomicAdd(&block_sums[r / 64u], static_cast<unsigned long long>(sz));
  });
  if (P.list) return;
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  unsigned long long v = (size & kSizeErr) ? 0ull : size;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const uint64_t blk = r / 64u;
  if (block_sums && (threadIdx.x & 63u) == 0 && blk * 64u < n) block_sums[blk] = v;
}

// The chain pass of the size walk (see "Chains"): the chains the main pass
// handed over, one wave each.  A node's events are the serial walk's: its
// first error in chain order, or xdr_overflow where the record's running
// size reaches kSizeErr first (the walk tests it after every field); a node
// that needs more frames than the registers hold, or a container of more
// than one element at a chain's link, sends the record to deep pass A, which
// walks it whole (its bytes so far taken back out of the block sum).
template <class OPS>
__device__ __forceinline__ void sub_chain_size_kernel(XDRG_SUB_SIZE_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  load_ops(sops, ops, nops);
  (void)mark;
  (void)depths;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nwv = static_cast<uint64_t>(gridDim.x) * (blockDim.x / 64u);
  const uint64_t nc = min(static_cast<uint64_t>(*P.chain_cnt), static_cast<uint64_t>(P.chain_cap));
  for (uint64_t c = static_cast<uint64_t>(blockIdx.x) * (blockDim.x / 64u) + (threadIdx.x >> 6); c < nc; c += nwv) {
    const sub_node h = P.heads[c];
    if (h.chain == ~0u) continue;  // logged by its lane
    const uint64_t r = P.chain_rec[c];
    const uint32_t part = sizes[r];
    const xdrg_op &v = sops[h.vpc];
    uint64_t eb = h.eb, start = h.s, k = 0;
    int64_t d = static_cast<int64_t>(v.arg1);  // the spacing guessed: the element size, then the one seen
    bool logged = true;
    int fate = 0;  // 1: closed, 2: an event (reported), 3: to deep pass A
    uint64_t total = 0;
    while (!fate) {
      const uint64_t a = eb + static_cast<uint64_t>(d * static_cast<int64_t>(lane));
      sub_src_t<OPS::kImgWords> src{native + r * stride, stride, heap, heap_len, a, true, {}};
      src.refresh();
      sub_size_node nd;
      nd.pc = v.arg4;
      nd.stop = h.vpc;
      nd.lf = h.chain + static_cast<uint32_t>(k) + lane;
      uint64_t sz = 0;
      uint32_t dmax = 0, bad_op = 0, code = 0;
      reg_stack st;
      chain_logger nolog{P, false, r};
      const int rc = sub_size<false, OPS, reg_stack, true>(sops, table, src, sz, dmax, bad_op, code, st, nolog, &nd);
      // the chain's nodes in this wave: lanes 0..J, each reached by the link before it
      const bool link = rc == kWalkOk && nd.cnt == 1u && nd.next == a + static_cast<uint64_t>(d);
      const uint64_t nl = __ballot(!link);
      const uint32_t J = nl ? static_cast<uint32_t>(__builtin_ctzll(nl)) : 63u;
      const bool mine = lane <= J;
      // first bytes: a prefix sum of the sizes (an error lane counts the bytes
      // before its failing field, for the overflow test below)
      const uint64_t w = !mine ? 0ull : rc == kWalkOk ? sz : rc == kWalkErr && sz >= 4 ? sz - 4 : 0ull;
      uint64_t incl = w;
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t x = __shfl_up(incl, o, 64);
        if (lane >= static_cast<uint32_t>(o)) incl += x;
      }
      const uint64_t first = start + incl - w;  // the node's first byte
      const bool over = mine && first + w >= kSizeErr;
      const bool event = mine && (over || rc == kWalkErr);
      const bool bail = mine && (rc == kWalkFull || (rc == kWalkOk && nd.cnt > 1u));
      const uint64_t em = __ballot(event), bm = __ballot(bail);
      const uint32_t E = em ? static_cast<uint32_t>(__builtin_ctzll(em)) : 64u;
      const uint32_t B = bm ? static_cast<uint32_t>(__builtin_ctzll(bm)) : 64u;
      if (E < 64u && E <= B) {
        if (lane == E) {
          if (over) report(err, r, 0, XDRG_ERR_OVERFLOW_PUT);
          else report(err, r, bad_op, code);
        }
        fate = 2;
        break;
      }
      if (B < 64u) {
        fate = 3;
        break;
      }
      // log lanes 0..J (a chunk of kChainChunk slots for the wave)
      if (logged) {
        unsigned long long at = 0;
        if (lane == 0) at = atomicAdd(P.node_cnt, static_cast<unsigned long long>(kChainChunk));
        at = __shfl(at, 0, 64);
        if (at + kChainChunk > P.node_cap) {
          logged = false;  // the log is full: the encode's walk writes this record whole
        } else {
          P.nodes[at + lane] = mine ? sub_node{a, static_cast<uint32_t>(first), h.dbase + static_cast<uint32_t>(k + lane) * v.depth,
                                               static_cast<uint32_t>(c), h.vpc}
                                    : sub_node{0, 0, 0, ~0u, 0};
        }
      }
      const uint64_t end = __shfl(first + sz, J, 64);  // past node J's count word
      const uint32_t cj = __shfl(nd.cnt, J, 64);
      const uint64_t nx = __shfl(nd.next, J, 64), aj = __shfl(a, J, 64);
      k += J + 1u;
      start = end;
      if (cj == 0u) {
        total = end;
        fate = 1;
      } else {
        d = static_cast<int64_t>(nx - aj);
        eb = nx;
      }
    }
    if (lane != 0) continue;
    const uint64_t blk = r / 64u;
    if (fate == 1) {
      sizes[r] = static_cast<uint32_t>(total);
      P.chain_end[c] = static_cast<uint32_t>(total);
      if (!logged) P.chain_of[r] = ~0u;
      if (block_sums) atomicAdd(&block_sums[blk], static_cast<unsigned long long>(total - part));
    } else {
      P.chain_of[r] = ~0u;
      if (block_sums) atomicAdd(&block_sums[blk], 0ull - static_cast<unsigned long long>(part));
      if (fate == 2) sizes[r] = kSizeErr;
      else P.defer[atomicAdd(P.defer_count, 1ull)] = static_cast<uint32_t>(r);
    }
  }
}

// -------------------------------------------------------------- encode
// Write combining of a lane's stream words: the stream's current 64-byte
// line in 16 words of LDS and a mask.  A line leaves when the walk moves
// past it: whole (four 16-byte stores) when the lane wrote all of it, else
// word by word (a record's first and last lines, shared with its
// neighbours).  Word stores straight from the walk left the lines half
// written in L2 between a lane's visits: rp_list's main encode pass wrote
// 1,434 MB to HBM per launch for 132 MB of stream, 1,030 µs; buffered, 695
// MB and 561 µs (profiles/r04y_pmc.json, r04af_pmc.json).  The deep passes
// (a few lanes, each walking a long chain serially) store directly: the
// buffer's LDS traffic lengthened their chains (3.5 -> 4.7 ms).
struct line_writer {
  uint32_t *buf;  // this lane's 16 words of LDS
  uint8_t *xdr;
  uint64_t ln;    // the buffered line: absolute address / 64
  uint32_t mask;
  bool on;        // false: every word straight to the stream
  __device__ __forceinline__ void flush() {
    if (!mask) return;
    uint8_t *g = reinterpret_cast<uint8_t *>(ln << 6);
    if (mask == 0xffffu) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<u32x4 *>(g + 16 * q) = *reinterpret_cast<const u32x4 *>(buf + 4 * q);
    } else {
      for (uint32_t m = mask; m; m &= m - 1u) {
        const uint32_t k = __builtin_ctz(m);
        st32(g + 4u * k, buf[k]);
      }
    }
    mask = 0;
  }
  __device__ __forceinline__ void put(uint64_t pos, uint32_t w) {
    if (!on) {
      st32(xdr + pos, w);
      return;
    }
    const uint64_t a = reinterpret_cast<uint64_t>(xdr) + pos;
    if ((a >> 6) != ln) {
      flush();
      ln = a >> 6;
    }
    const uint32_t k = static_cast<uint32_t>(a >> 2) & 15u;
    buf[k] = w;
    mask |= 1u << k;
  }
};

// The node pass writes a logged chain only where no field of the record can
// fail (it fits `cap`, no stack limit): its lanes then report nothing, and a
// record that can fail is walked whole, its error the reference's first.
__device__ __forceinline__ bool sub_chain_writes(uint64_t off, uint32_t sz, uint64_t cap, uint32_t stack_limit) {
  return off + sz <= cap && stack_limit == 0xffffffffu;
}

// Where an encode walk starts: the record from its first op (the
// defaults), or a logged chain node (the node pass: its element in src,
// record-relative byte `rel`, its body's first op and depth base, ending at
// its chain's count word, op `stop`).  chain_end: where the record's logged
// chain closes (record-relative; ~0: not logged), for the main pass.
struct sub_start {
  uint32_t pc = 0, dbase = 0, stop = ~0u, chain_end = ~0u;
  uint64_t rel = 0;
};

// The record's walk from stream offset `off` with check(n) and the stack
// budget before every field (marshal.h:104-108, :129-136).  Errors are
// reported; kWalkFull when the stack ran out (op in *full_op).
template <class OPS, class ST>
__device__ __forceinline__ int sub_encode_rec(const xdrg_op *__restrict__ sops, const uint32_t *__restrict__ table,
                              sub_src_t<OPS::kImgWords> src,
                              line_writer &lw, uint64_t cap, uint64_t off, uint32_t sz, uint32_t mark,
                              uint32_t stack_limit, uint64_t r, unsigned long long *err, uint32_t *full_op,
                              ST &st, const sub_start &at = sub_start{}) {
  const uint8_t *heap = src.heap;
  const uint64_t heap_len = src.heap_len;
  uint64_t pos = off + at.rel;
  if (mark && !at.rel) {  // the message's record mark (message_t::alloc, marshal.cc:15-31)
    if (4 > cap - min(pos, cap)) { report(err, r, kOpRecordLevel, XDRG_ERR_OVERFLOW_PUT); return kWalkErr; }
    lw.put(pos, mark_word(sz - 4u));
    pos += 4;
  }
  uint32_t fp = 0, pc = at.pc, dbase = at.dbase;
  bool skipped = false;  // the record's first chain past kChainT was met
  st.lf = 0;
  auto step = [&](const auto &op) __attribute__((always_inline)) -> int {
    if (op.kind == XDRG_OP_END) {
      if (!sub_next(sops, st, fp, pc, dbase, src.eb, src.in_heap)) return kWalkOk;
      src.refresh();
      return kWalkCont;
    }
    if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; return kWalkCont; }
    if (dbase + op.depth > stack_limit) { report(err, r, pc, XDRG_ERR_STACK_PUT); return kWalkErr; }
    uint64_t need = 4;
    uint32_t len = 0;
    if (op.kind == XDRG_OP_U64) need = 8;
    else if (op.kind == XDRG_OP_OPAQUE) need = op.arg0;
    else if (op.kind == XDRG_OP_VAROPAQUE || op.kind == XDRG_OP_STRING) {
      len = src.w(op.noff + 8);
      need = 4ull + len;
    }
    if (need > cap - min(pos, cap)) { report(err, r, pc, XDRG_ERR_OVERFLOW_PUT); return kWalkErr; }
    const uint64_t p0 = pos;  // the field's first stream byte
    switch (op.kind) {
    case XDRG_OP_U32: case XDRG_OP_ENUM: lw.put(p0, bswap32(src.w(op.noff))); pos += 4; ++pc; break;
    case XDRG_OP_BOOL: lw.put(p0, src.b(op.noff) ? 0x01000000u : 0u); pos += 4; ++pc; break;
    case XDRG_OP_U64:
      lw.put(p0, bswap32(src.w(op.noff + 4)));
      lw.put(p0 + 4, bswap32(src.w(op.noff)));
      pos += 8;
      ++pc;
      break;
    case XDRG_OP_OPAQUE: {
      const uint32_t L = op.arg0, nw = (L + 3u) >> 2;
      for (uint32_t k = 0; k < nw; ++k) {
        uint32_t w = src.wu(op.noff + 4u * k);
        if (4 * k + 4 > L) w &= keep_mask(L - 4 * k);
        lw.put(p0 + 4ull * k, w);
      }
      pos += 4ull * nw;
      ++pc;
      break;
    }
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      const uint64_t hoff = src.w64(op.noff);
      const uint32_t nw = (len + 3u) >> 2;
      lw.put(p0, bswap32(len));
      for (uint32_t k = 0; k < nw; k += 4) {  // four words' loads at a time
        uint32_t w[4];
        src.hwords4(hoff + 4ull * k, w);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          if (k + j >= nw) break;
          uint32_t x = w[j];
          if (4 * (k + j) + 4 > len) x &= keep_mask(len - 4 * (k + j));
          lw.put(p0 + 4ull + 4ull * (k + j), x);
        }
      }
      pos += 4ull + 4ull * nw;
      ++pc;
      break;
    }
    case XDRG_OP_UNION: {
      const uint32_t d = src.w(op.noff);
      lw.put(p0, bswap32(d));
      pos += 4;
      pc = static_cast<uint32_t>(union_target(op, table, d));  // validated by the size pass
      break;
    }
    case XDRG_OP_VECTOR: {
      const uint64_t eoff = src.w64(op.noff);
      const uint32_t cnt = src.w(op.noff + 8);
      lw.put(p0, bswap32(cnt));
      pos += 4;
      if (!(op.flags & XDRG_F_SUB)) {
        uint32_t at = static_cast<uint32_t>(pos - off);
        auto put = [&](uint32_t a, uint32_t w) { lw.put(off + a, w); };
        if (!enc_vector_elems(sops, pc + 1, op.arg2, heap, heap_len, eoff, cnt, op.arg1, pos, cap, at,
                              stack_limit - dbase, r, err, put))
          return kWalkErr;
        pc += 1 + op.arg2;
        break;
      }
      if (fp == 0 && pc == at.stop) return kWalkOk;  // a logged node ends with its chain's count word
      if (!cnt) { ++pc; break; }
      if (!skipped && fp && st.top(fp).left == 0u && st.top(fp).nf == kChainT && st.lf < XDRG_MAX_FRAMES &&
          sub_tail(sops, pc)) {
        // the record's first chain this long (the size walk's chain_logger
        // met it here): logged, the node pass writes it from here on, and
        // the walk goes on where the chain closes, its frame popped
        skipped = true;
        if (at.chain_end != ~0u) {
          const sub_frame t = st.top(fp);
          pc = t.ret();
          dbase -= t.dsum;
          st.lf -= t.nf;
          st.pop(fp);
          if (--fp) src.eb = st.top(fp).eb;
          else src.in_heap = false;
          src.refresh();
          pos = off + at.chain_end;
          break;
        }
      }
      bool tail = false;
      const int o = sub_open(sops, st, fp, pc, op.depth, eoff, cnt, true, &tail);
      if (o == kOpenFull) { *full_op = pc; return kWalkFull; }
      if (o == kOpenOver) { report(err, r, pc, XDRG_ERR_STACK_PUT); return kWalkErr; }
      dbase += op.depth;
      src.eb = eoff;
      src.in_heap = true;
      src.refresh();
      pc = op.arg4;
      break;
    }
    default: ++pc; break;
    }
    return kWalkCont;
  };
  for (;;) {
    const int rc = OPS::visit(sops, pc, step);
    if (rc != kWalkCont) return rc;
  }
}

// Record offsets as k_var_encode computes them (block-local scan on top of
// the 64-record block bases); a deep pass reads them back.
template <class OPS>
__device__ __forceinline__ void sub_encode_kernel(XDRG_SUB_ENCODE_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  load_ops(sops, ops, nops);
  uint64_t off = 0;
  if (!P.list) {
    const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint32_t sz = r < n ? sizes[r] : 0u;
    const unsigned long long v = (sz & kSizeErr) ? 0ull : sz;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long incl = v;
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long x = __shfl_up(incl, o, 64);
      if (lane >= static_cast<uint32_t>(o)) incl += x;
    }
    if (r >= n) return;
    off = block_base[blockIdx.x * 4u + wid] + incl - v;
    offsets[r] = off;
  }
  // after the ops (host: + 64 B a lane for the line writer)
  line_writer lw{smem + 8u * nops + 16u * threadIdx.x, xdr, ~0ull, 0u, !P.list && P.lines != 0};
  sub_records(P, n, [&](uint64_t r, auto &st) {
    const uint32_t sz = sizes[r];
    if (sz & kSizeErr) return;  // the size pass reported this record
    const uint64_t o = P.list ? offsets[r] : off;
    const sub_src_t<OPS::kImgWords> src{native + r * stride, stride, heap, heap_len, 0, false, {}};
    uint32_t full_op = 0;
    sub_start at;
    if (!P.list && P.chain_of && sub_chain_writes(o, sz, cap, stack_limit)) {
      const uint32_t c = P.chain_of[r];  // the record's logged chain, if any: the node pass writes it
      if (c != ~0u) at.chain_end = P.chain_end[c];
    }
    const int rc = sub_encode_rec<OPS>(sops, table, src, lw, cap, o, sz, mark, stack_limit, r, err, &full_op, st, at);
    lw.flush();
    if (rc == kWalkFull) sub_full(P, r, full_op, XDRG_ERR_STACK_PUT, err);
  });
}

// The node pass (see "Chains"): every node the size walks logged, one lane
// each, written from its element to its chain's count word at its place in
// its record's stretch (the main pass wrote the record's offset).  A
// record whose size walk failed is skipped; a node of a record whose main
// pass deferred it, or whose chain was not logged to its close, writes the
// bytes the record's own walk writes too.
template <class OPS>
__device__ __forceinline__ void sub_chain_kernel(XDRG_SUB_ENCODE_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  load_ops(sops, ops, nops);
  (void)block_base;
  (void)mark;
  const uint64_t total = min(static_cast<uint64_t>(*P.node_cnt), static_cast<uint64_t>(P.node_cap));
  const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  line_writer lw{nullptr, xdr, ~0ull, 0u, false};
  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < total; k += lanes) {
    const sub_node e = P.nodes[k];
    if (e.chain >= P.chain_cap) continue;  // an unused slot
    const uint64_t r = P.chain_rec[e.chain];
    if (r >= n) continue;
    const uint32_t sz = sizes[r];
    if ((sz & kSizeErr) || !sub_chain_writes(offsets[r], sz, cap, stack_limit)) continue;
    sub_src_t<OPS::kImgWords> src{native + r * stride, stride, heap, heap_len, e.eb, true, {}};
    src.refresh();
    sub_start at;
    at.pc = sops[e.vpc].arg4;
    at.dbase = e.dbase;
    at.stop = e.vpc;
    at.rel = e.s;
    reg_stack st;
    uint32_t full_op = 0;
    // (a node nested past the main pass's frames belongs to a record the deep
    // passes write whole: kWalkFull needs nothing here)
    (void)sub_encode_rec<OPS>(sops, table, src, lw, cap, offsets[r], sz, 0u, stack_limit, r, err, &full_op, st, at);
  }
}

// -------------------------------------------------------------- decode
// Record r = xdr_from_opaque(stream[a, b), r) with check(n) before every
// read; the native record and every element array are zero-filled first.
// Payloads stay in the stream (heap_out holds it at [0, len)); element
// arrays come from the record's element area [ecur, eend) at 8-byte
// alignment.  On a failure inside elements, each open container's rsv
// holds 1 + the index of the element that failed, the others 0 (the
// unstager follows these marks).  kWalkFull: the stack ran out (op in
// *full_op), nothing reported.  The stream's words come through rd
// (glob_rd, or the wave pass's wave_rd).
template <class OPS, class ST, class RD>
__device__ __forceinline__ int sub_decode_rec(const xdrg_op *__restrict__ sops, const uint32_t *__restrict__ table,
                              const uint8_t *__restrict__ xdr, uint64_t a, uint64_t b, uint8_t *__restrict__ rec,
                              uint32_t stride, uint8_t *__restrict__ heap, uint64_t ecur, uint64_t eend,
                              uint32_t stack_limit, uint64_t r, unsigned long long *err, uint32_t *full_op,
                              ST &st, bool defer, const RD &rd) {
  zero_words<RD>(rec, stride & ~3u);
  uint64_t p = a;
  // (The stream through a 32-byte read-ahead, two aligned 16-byte chunks
  // serving up to 8 words per round trip, measured slower: rp_list's decode
  // 3.94 vs 2.76 ms, profiles/r05o.)
  auto word = [&](uint64_t q) -> uint32_t { return rd(q); };
  uint32_t fp = 0, pc = 0, dbase = 0, code = 0;
  st.lf = 0;
  uint64_t eb = 0;
  bool in_heap = false;
  // Tail containers replace frames only where a record whose walk fails can
  // be deferred to a deep pass that does not (the failing element's marks
  // go in every open container, replaced ones too): recursive plans' main
  // pass.
  const bool may_tail = ST::kRegs && defer;
  bool tailed = false;
  auto step = [&](const auto &op) __attribute__((always_inline)) -> int {
    if (op.kind == XDRG_OP_END) return sub_next(sops, st, fp, pc, dbase, eb, in_heap) ? kWalkCont : kWalkOk;
    if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; return kWalkCont; }
    if (dbase + op.depth > stack_limit) { code = XDRG_ERR_STACK_GET; return kWalkErr; }
    uint8_t *nat = in_heap ? heap + eb : rec;
    const uint64_t rem = b - p;
    switch (op.kind) {
    case XDRG_OP_U32:
      if (rem < 4) { code = XDRG_ERR_OVERFLOW_GET; break; }
      st32(nat + op.noff, bswap32(word(p))); p += 4; ++pc; break;
    case XDRG_OP_ENUM: {
      if (rem < 4) { code = XDRG_ERR_OVERFLOW_GET; break; }
      const uint32_t v = bswap32(word(p));
      st32(nat + op.noff, v); p += 4;
      if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, v)) { code = XDRG_ERR_INVALID_ENUM; break; }
      ++pc; break;
    }
    case XDRG_OP_BOOL:
      if (rem < 4) { code = XDRG_ERR_OVERFLOW_GET; break; }
      nat[op.noff] = word(p) != 0u; p += 4; ++pc; break;
    case XDRG_OP_U64:
      if (rem < 8) { code = XDRG_ERR_OVERFLOW_GET; break; }
      st32(nat + op.noff + 4, bswap32(word(p)));
      st32(nat + op.noff, bswap32(word(p + 4)));
      p += 8; ++pc; break;
    case XDRG_OP_OPAQUE: {
      const uint32_t L = op.arg0;
      if (rem < L) { code = XDRG_ERR_OVERFLOW_GET; break; }
      if constexpr (RD::kWave) {
        for (uint32_t q = 0; q < L; q += 4) {
          const uint32_t w = word(p + q);
          for (uint32_t k = 0; k < 4u && q + k < L; ++k) nat[op.noff + q + k] = uint8_t(w >> (8u * k));
        }
      } else {
        for (uint32_t k = 0; k < L; ++k) nat[op.noff + k] = xdr[p + k];
      }
      if ((L & 3u) && (word(p + (L & ~3u)) & ~keep_mask(L & 3u))) { code = XDRG_ERR_NONZERO_PAD; break; }
      p += (L + 3u) & ~3u; ++pc; break;
    }
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      if (rem < 4) { code = XDRG_ERR_OVERFLOW_GET; break; }
      const uint32_t L = bswap32(word(p));
      if (L > rem - 4) { code = XDRG_ERR_OVERFLOW_GET; break; }
      if (L > op.arg0) { code = op.kind == XDRG_OP_STRING ? XDRG_ERR_XSTRING_BOUND : XDRG_ERR_XVECTOR_BOUND; break; }
      p += 4;
      const uint32_t nw = (L + 3u) >> 2;
      if ((L & 3u) && (word(p + 4ull * (nw - 1)) & ~keep_mask(L & 3u))) { code = XDRG_ERR_NONZERO_PAD; break; }
      *reinterpret_cast<uint64_t *>(nat + op.noff) = p;  // the payload stays in the stream
      st32(nat + op.noff + 8, L);
      p += 4ull * nw; ++pc; break;
    }
    case XDRG_OP_UNION: {
      if (rem < 4) { code = XDRG_ERR_OVERFLOW_GET; break; }
      const uint32_t d = bswap32(word(p));
      p += 4;
      if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, d)) { code = XDRG_ERR_INVALID_ENUM; break; }
      const int t = union_target(op, table, d);
      if (t < 0) { code = XDRG_ERR_BAD_DISCRIMINANT; break; }
      st32(nat + op.noff, d);
      pc = static_cast<uint32_t>(t);
      break;
    }
    case XDRG_OP_VECTOR: {
      if (rem < 4) { code = XDRG_ERR_OVERFLOW_GET; break; }
      const uint32_t cnt = bswap32(word(p));
      p += 4;
      if (cnt > op.arg0) {  // check_size (types.h:486-489, 605-608)
        code = (op.flags & XDRG_F_POINTER) ? XDRG_ERR_POINTER_BOUND : XDRG_ERR_XVECTOR_BOUND;
        break;
      }
      // Element area.  Valid data never overruns it (distinct elements
      // start at distinct wire words, include/xdrgpu.h heap factor); a
      // forged count could, so every reservation is checked.  Every element
      // takes at least arg3 wire bytes (the inline element size, or the
      // least an element subroutine consumes): an element subroutine's count
      // the bytes left cannot hold fails here, before any area is reserved,
      // with the xdr_overflow the reference raises at the element that runs
      // out; inline elements fail at that element, so only the ones that
      // can be reached are reserved.
      const uint64_t bytes = static_cast<uint64_t>(cnt) * op.arg1;
      const uint64_t reach = (op.flags & XDRG_F_SUB)
                                 ? bytes
                                 : min(static_cast<uint64_t>(cnt), (b - p) / op.arg3 + 1) * op.arg1;
      ecur = (ecur + 7u) & ~7ull;
      if (((op.flags & XDRG_F_SUB) && static_cast<uint64_t>(cnt) * op.arg3 > b - p) || ecur > eend ||
          reach > eend - ecur) {
        code = XDRG_ERR_OVERFLOW_GET;
        break;
      }
      *reinterpret_cast<uint64_t *>(nat + op.noff) = ecur;
      st32(nat + op.noff + 8, cnt);
      if (!(op.flags & XDRG_F_SUB)) {
        auto rd = [&](uint64_t q) { return word(q); };
        if (!dec_vector_elems(sops, table, pc + 1, op.arg2, cnt, op.arg1, heap + ecur, p, b,
                              stack_limit - dbase, r, err, rd, reinterpret_cast<uint32_t *>(nat + op.noff + 12))) {
          code = kReported;
          break;
        }
        ecur += bytes;
        pc += 1 + op.arg2;
        break;
      }
      if (!cnt) { ++pc; break; }
      const int o = sub_open(sops, st, fp, pc, op.depth, ecur, cnt, may_tail, &tailed);
      if (o == kOpenFull) { *full_op = pc; return kWalkFull; }
      if (o == kOpenOver) { code = XDRG_ERR_STACK_GET; break; }
      uint8_t *arr = heap + ecur;
      zero_words<RD>(arr, bytes & ~3ull);
      for (uint64_t z = bytes & ~3ull; z < bytes; ++z) arr[z] = 0;
      dbase += op.depth;
      eb = ecur;
      in_heap = true;
      ecur += bytes;
      pc = op.arg4;
      break;
    }
    default: ++pc; break;
    }
    return code ? kWalkErr : kWalkCont;
  };
  int rc;
  do rc = OPS::visit(sops, pc, step);
  while (rc == kWalkCont);
  if (rc == kWalkFull) return kWalkFull;
  if (code && tailed) {  // the deep pass walks it again with every frame
    *full_op = pc;
    return kWalkFull;
  }
  if (code) {
    if (code != kReported) report(err, r, pc, code);
    // 1 + the failing element in every open container: the container's ref
    // sits in the object that encloses it (the record, or the frame below)
    st.each(fp, [&](uint32_t k, const sub_frame &fk, const sub_frame &below) {
      uint8_t *ref = (k ? heap + below.eb : rec) + sops[fk.vpc()].noff;
      st32(ref + 12, ld32(ref + 8) - fk.left);
    });
    return kWalkErr;
  }
  if (p != b) report(err, r, kOpRecordLevel, XDRG_ERR_TRAILING);
  return kWalkOk;
}

// Packed element areas (oracle/xdr_oracle.c rec_ebytes): the bytes the
// element arrays of the record at [p, b) take, each rounded up to 8 -- a
// walk of its lengths, counts and discriminants (no value checks) that
// stops where the structure stops parsing.  An element subroutine's array
// counts when the bytes left can hold its count (arg3 = the least an
// element consumes), then its elements' own arrays.  Non-recursive plans
// only (packed): kSubFrames frames always suffice.
__device__ uint64_t sub_ebytes(const xdrg_op *__restrict__ ops, const uint32_t *__restrict__ table,
                               const uint8_t *__restrict__ xdr, uint64_t p, uint64_t b) {
  uint32_t left[kSubFrames], vpc[kSubFrames];
  uint32_t fp = 0, pc = 0;
  uint64_t E = 0;
  for (;;) {
    const xdrg_op &op = ops[pc];
    if (op.kind == XDRG_OP_END) {
      if (!fp) return E;
      if (left[fp - 1]) { --left[fp - 1]; pc = ops[vpc[fp - 1]].arg4; }
      else pc = vpc[--fp] + 1;
      continue;
    }
    if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; continue; }
    const uint64_t rem = b - p;
    switch (op.kind) {
    case XDRG_OP_U64: if (rem < 8) return E; p += 8; ++pc; continue;
    case XDRG_OP_OPAQUE: if (rem < op.arg0) return E; p += (op.arg0 + 3u) & ~3u; ++pc; continue;
    case XDRG_OP_U32: case XDRG_OP_BOOL: case XDRG_OP_ENUM: if (rem < 4) return E; p += 4; ++pc; continue;
    default: break;
    }
    if (rem < 4) return E;
    const uint32_t v = bswap32(ld32(xdr + p));
    p += 4;
    const uint64_t lft = b - p;
    switch (op.kind) {
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
      if (v > op.arg0 || v > lft) return E;
      p += (static_cast<uint64_t>(v) + 3u) & ~3ull;
      ++pc;
      break;
    case XDRG_OP_UNION: {
      const int t = union_target(op, table, v);
      if (t < 0) return E;
      pc = static_cast<uint32_t>(t);
      break;
    }
    case XDRG_OP_VECTOR:
      if (v > op.arg0) return E;
      if (op.flags & XDRG_F_SUB) {
        if (lft < static_cast<uint64_t>(v) * op.arg3) return E;
        E += (static_cast<uint64_t>(v) * op.arg1 + 7u) & ~7ull;
        if (!v) { ++pc; break; }
        if (fp == kSubFrames) return E;  // (a packed plan never nests this deep)
        left[fp] = v - 1;
        vpc[fp++] = pc;
        pc = op.arg4;
        break;
      }
      E += (min<uint64_t>(v, lft / op.arg3 + 1u) * op.arg1 + 7u) & ~7ull;
      if (lft < static_cast<uint64_t>(v) * op.arg3) return E;
      p += static_cast<uint64_t>(v) * op.arg3;
      pc += 1 + op.arg2;
      break;
    default: ++pc; break;
    }
  }
}

// Linked lists in the wave pass.  A plan that is one node of a list -- flat
// fields, then an optional pointer to its own type as the last field, the
// RPCBPROC_DUMP reply's rp__list (xdrpp/rpcb_prot.x:32-37) -- decodes a long
// record a batch of up to 64 nodes at a time instead of a node per step of
// the whole wave: the wave walks the nodes' lengths and counts alone, in step
// (scalar, from the LDS block: each node's first byte and element area, and
// every check the walk makes on them), then each lane decodes one node of
// the batch from the block, the value checks first (pads, enums) and the
// batch written only when all its nodes pass.  A record that leaves that
// shape (a failed check, a node longer than the block, trailing bytes) goes
// to the walk from its start (false), which writes again every node the
// batches wrote, since they all come before its failure.
__device__ __forceinline__ bool flat_kind(uint32_t k) {
  return k == XDRG_OP_U32 || k == XDRG_OP_U64 || k == XDRG_OP_BOOL || k == XDRG_OP_ENUM ||
         k == XDRG_OP_OPAQUE || k == XDRG_OP_VAROPAQUE || k == XDRG_OP_STRING;
}
// The list's VECTOR op, or ~0u when the plan is not one node of a list.
__device__ __forceinline__ uint32_t list_vpc(const xdrg_op *__restrict__ ops, uint32_t nops) {
  uint32_t pc = 0;
  while (pc < nops && flat_kind(ops[pc].kind)) ++pc;
  if (pc == 0 || pc >= nops) return ~0u;
  const xdrg_op &v = ops[pc];
  constexpr uint32_t kPtr = XDRG_F_SUB | XDRG_F_POINTER;
  if (v.kind != XDRG_OP_VECTOR || (v.flags & kPtr) != kPtr || v.arg0 != 1u || v.arg4 != 0u || !v.arg3)
    return ~0u;
  return sub_tail(ops, pc) ? pc : ~0u;
}

template <class OPS>
__device__ __forceinline__ bool list_decode(const xdrg_op *__restrict__ sops, uint32_t vpc,
                                         const uint32_t *__restrict__ table, const uint8_t *__restrict__ xdr,
                                         uint64_t a, uint64_t b, uint8_t *__restrict__ rec, uint32_t stride,
                                         uint8_t *__restrict__ heap, uint64_t ecur, uint64_t eend,
                                         uint32_t stack_limit, uint32_t *blk, uint16_t *nxt) {
  const uint32_t lane = threadIdx.x & 63u;
  const xdrg_op &V = sops[vpc];
  const uint32_t vdepth = V.depth, esz = V.arg1, emin = V.arg3, vnoff = V.noff;
  uint32_t maxd = 0;
  for (uint32_t q = 0; q <= vpc; ++q) maxd = max(maxd, static_cast<uint32_t>(sops[q].depth));
  uint64_t base = ~0ull;  // stream offset of blk[0]
  auto load = [&](uint64_t q) {
    const uint64_t b0 = q & ~15ull;
    wave_sync();  // every lane past its reads of the old block
    // (all eight loads in flight before the stores took 27 more VGPRs in a
    // kernel the main pass shares)
    for (uint32_t j = 0; j < kWaveBlk / 1024u; ++j) {
      const uint32_t k = lane + 64u * j;
      const uint64_t o = b0 + 16ull * k;
      u32x4 v{0u, 0u, 0u, 0u};
      if (o + 16 <= b) {
        v = ld16u(xdr + o);
      } else if (o < b) {
        v.x = ld32(xdr + o);
        if (o + 8 <= b) v.y = ld32(xdr + o + 4);
        if (o + 12 <= b) v.z = ld32(xdr + o + 8);
      }
      *reinterpret_cast<u32x4 *>(blk + 4u * k) = v;
    }
    wave_sync();
    base = b0;
    if (!nxt) return;
    // every word of the block as a node start, a lane two words at a time
    // (their LDS reads in flight together): the node's words and its
    // pointer's count, (words << 1 | count), or 0 where a check fails or a
    // read leaves the block.  The chain from the record's first byte meets
    // only true node starts, so it follows these in one LDS read a node (a 0
    // on it: the scalar walk below takes that node).
    constexpr uint32_t kHalf = kWaveBlk / 8u;  // words per cursor
    for (uint32_t w = lane; w < kHalf; w += 64u) {
      uint64_t c[2] = {b0 + 4ull * w, b0 + 4ull * (w + kHalf)};
      const uint64_t q[2] = {c[0], c[1]};
      bool live[2] = {q[0] < b, q[1] < b};
      uint32_t cn[2] = {0u, 0u};
      if (live[0] || live[1]) {
        uint32_t pc = 0;
        auto cand = [&](const auto &op) __attribute__((always_inline)) -> int {
#pragma unroll
          for (uint32_t i = 0; i < 2; ++i) {
            const uint64_t rem = b - c[i];
            bool ok = live[i];
            switch (op.kind) {
            case XDRG_OP_U32: case XDRG_OP_BOOL: case XDRG_OP_ENUM:
              ok = ok && rem >= 4;
              c[i] += 4; break;
            case XDRG_OP_U64:
              ok = ok && rem >= 8;
              c[i] += 8; break;
            case XDRG_OP_OPAQUE:
              ok = ok && rem >= op.arg0;
              c[i] += (op.arg0 + 3u) & ~3u; break;
            case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
              ok = ok && rem >= 4 && c[i] - b0 < kWaveBlk;
              const uint32_t L = ok ? bswap32(blk[(c[i] - b0) >> 2]) : 0u;
              ok = ok && L <= rem - 4 && L <= op.arg0;
              c[i] += 4 + 4ull * ((L + 3u) >> 2); break;
            }
            default:
              ok = ok && rem >= 4 && c[i] - b0 < kWaveBlk;
              cn[i] = ok ? bswap32(blk[(c[i] - b0) >> 2]) : 0u;
              c[i] += 4;
              break;
            }
            live[i] = ok;
          }
          if (op.kind == XDRG_OP_VECTOR) return 0;
          if (!live[0] && !live[1]) return 1;
          ++pc;
          return kWalkCont;
        };
        int rc;
        do rc = OPS::visit(sops, pc, cand);
        while (rc == kWalkCont);
      }
#pragma unroll
      for (uint32_t i = 0; i < 2; ++i) {
        const bool ok = live[i] && cn[i] <= 1u && static_cast<uint64_t>(cn[i]) * emin <= b - c[i];
        nxt[w + i * kHalf] = static_cast<uint16_t>(ok ? static_cast<uint32_t>((c[i] - q[i]) >> 1) | cn[i] : 0u);
      }
    }
    wave_sync();
  };
  // the batch: lane j holds node k - nb + j's first byte, record-relative,
  // or'ed with its pointer's count.  Every pointer but the last holds one
  // element, so node k's pointer gets the area ref0 + k * align8(esz) (the
  // walk's bump pointer: aligned to 8, then one element on) and node k >= 1
  // is the element its predecessor's pointer got.
  uint32_t m_pc = 0, nb = 0, k = 0;  // k: the next node (0: the record)
  const uint64_t ref0 = (ecur + 7u) & ~7ull, esz8 = (static_cast<uint64_t>(esz) + 7u) & ~7ull;
#ifdef XDRG_LIST_STAMPS
  uint64_t ts_val = 0, ts_wr = 0, ts_ld = 0, ts_all = clock64(), n_fl = 0, n_ld = 0;
#define XLS(v, t) (v) += clock64() - (t)
#else
#define XLS(v, t) ((void)0)
#endif
  // lane decode of the batch from the block: checks, then (all pass) writes
  auto flush = [&]() -> bool {
    if (!nb) return true;
#ifdef XDRG_LIST_STAMPS
    uint64_t t0 = clock64(); ++n_fl;
#endif
    const bool on = lane < nb;
    const uint32_t kk = k - nb + lane, cnt = m_pc & 1u;
    const uint64_t ref = ref0 + static_cast<uint64_t>(kk) * esz8;
    uint64_t p = a + (m_pc & ~3u);
    auto wd = [&](uint64_t q) -> uint32_t { return blk[(q - base) >> 2]; };
    // the walk's checks on the node's depth, frames and element area, then
    // its pads and enums
    bool bad = on && (static_cast<uint64_t>(kk) * vdepth + maxd > stack_limit ||
                      (cnt && kk + 1u >= XDRG_MAX_FRAMES) || ref > eend ||
                      static_cast<uint64_t>(cnt) * esz > eend - ref);
    if (on) {
      uint32_t pc = 0;
      auto check = [&](const auto &op) __attribute__((always_inline)) -> int {
        switch (op.kind) {
        case XDRG_OP_U32: case XDRG_OP_BOOL: p += 4; break;
        case XDRG_OP_ENUM:
          if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, bswap32(wd(p)))) bad = true;
          p += 4; break;
        case XDRG_OP_U64: p += 8; break;
        case XDRG_OP_OPAQUE: {
          const uint32_t L = op.arg0;
          if ((L & 3u) && (wd(p + (L & ~3u)) & ~keep_mask(L & 3u))) bad = true;
          p += (L + 3u) & ~3u; break;
        }
        case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
          const uint32_t L = bswap32(wd(p));
          p += 4;
          const uint32_t nw = (L + 3u) >> 2;
          if ((L & 3u) && (wd(p + 4ull * (nw - 1)) & ~keep_mask(L & 3u))) bad = true;
          p += 4ull * nw; break;
        }
        default: return kWalkOk;  // the list's VECTOR
        }
        ++pc;
        return kWalkCont;
      };
      while (OPS::visit(sops, pc, check) == kWalkCont) {}
    }
    if (__any(bad)) return false;
    XLS(ts_val, t0);
#ifdef XDRG_LIST_STAMPS
    t0 = clock64();
#endif
    if (on) {
      uint8_t *nat = kk ? heap + (ref - esz8) : rec;
      if (!kk) {
        for (uint32_t z = 0; z + 4 <= stride; z += 4) st32(nat + z, 0u);
      } else {
        for (uint32_t z = 0; z + 4 <= esz; z += 4) st32(nat + z, 0u);
        for (uint32_t z = esz & ~3u; z < esz; ++z) nat[z] = 0;
      }
      p = a + (m_pc & ~3u);
      uint32_t pc = 0;
      auto put = [&](const auto &op) __attribute__((always_inline)) -> int {
        switch (op.kind) {
        case XDRG_OP_U32: case XDRG_OP_ENUM: st32(nat + op.noff, bswap32(wd(p))); p += 4; break;
        case XDRG_OP_BOOL: nat[op.noff] = wd(p) != 0u; p += 4; break;
        case XDRG_OP_U64:
          st32(nat + op.noff + 4, bswap32(wd(p)));
          st32(nat + op.noff, bswap32(wd(p + 4)));
          p += 8; break;
        case XDRG_OP_OPAQUE: {
          const uint32_t L = op.arg0;
          for (uint32_t q = 0; q < L; q += 4) {
            const uint32_t w = wd(p + q);
            for (uint32_t k = 0; k < 4u && q + k < L; ++k) nat[op.noff + q + k] = uint8_t(w >> (8u * k));
          }
          p += (L + 3u) & ~3u; break;
        }
        case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
          const uint32_t L = bswap32(wd(p));
          p += 4;
          *reinterpret_cast<uint64_t *>(nat + op.noff) = p;
          st32(nat + op.noff + 8, L);
          p += 4ull * ((L + 3u) >> 2); break;
        }
        default: return kWalkOk;
        }
        ++pc;
        return kWalkCont;
      };
      while (OPS::visit(sops, pc, put) == kWalkCont) {}
      *reinterpret_cast<uint64_t *>(nat + vnoff) = ref;
      st32(nat + vnoff + 8, cnt);
    }
    nb = 0;
    XLS(ts_wr, t0);
    return true;
  };
  // the list's end: the record's own END follows
  auto finish = [&](uint64_t p) -> bool {
    if (p != b) return false;
    const bool fin = flush();
#ifdef XDRG_LIST_STAMPS
    if (!lane) printf("LIST nodes %u flushes %lu loads %lu all %lu val %lu wr %lu ld %lu\n", k, n_fl, n_ld,
                      clock64() - ts_all, ts_val, ts_wr, ts_ld);
#endif
    return fin;
  };
  uint64_t p = a;
  for (;;) {
    if (base == ~0ull) {
#ifdef XDRG_LIST_STAMPS
      const uint64_t t0 = clock64(); ++n_ld;
#endif
      load(p);
      XLS(ts_ld, t0);
    }
    if (nxt) {  // the chain through the candidates: one LDS read a node
      uint32_t rel = static_cast<uint32_t>(p - a), off = static_cast<uint32_t>(p - base), e = 1u;
      while (nb < 64u && off < kWaveBlk) {
        e = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(nxt[off >> 2]));
        if (!e) break;
        m_pc = lane == nb ? rel | (e & 1u) : m_pc;
        ++nb;
        ++k;
        rel += 2u * (e & ~1u);
        off += 2u * (e & ~1u);
        if (!(e & 1u)) break;
      }
      p = a + rel;
      if (e && !(e & 1u)) return finish(p);
      if (nb == 64u) {
        if (!flush()) return false;
        continue;
      }
    }
    // the node's lengths and counts: its candidate, or scalar (0 its
    // pointer's count word read, 1 a check failed, 2 a read past the block)
    const uint64_t p0 = p;
    uint32_t cnt = 0;
    int rc = 0;
    const uint32_t e = nxt && p - base < kWaveBlk
                           ? __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(nxt[(p - base) >> 2]))
                           : 0u;
    if (e) {  // the candidate pass's node
      cnt = e & 1u;
      p += 2ull * (e & ~1u);
    } else {
      uint32_t pc = 0;
      auto skel = [&](const auto &op) __attribute__((always_inline)) -> int {
        const uint64_t rem = b - p;
        switch (op.kind) {
        case XDRG_OP_U32: case XDRG_OP_BOOL: case XDRG_OP_ENUM:
          if (rem < 4) return 1;
          p += 4; break;
        case XDRG_OP_U64:
          if (rem < 8) return 1;
          p += 8; break;
        case XDRG_OP_OPAQUE:
          if (rem < op.arg0) return 1;
          p += (op.arg0 + 3u) & ~3u; break;
        case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
          if (rem < 4) return 1;
          if (p - base >= kWaveBlk) return 2;
          const uint32_t L = bswap32(__builtin_amdgcn_readfirstlane(blk[(p - base) >> 2]));
          if (L > rem - 4 || L > op.arg0) return 1;
          p += 4 + 4ull * ((L + 3u) >> 2); break;
        }
        default:  // the list's VECTOR: its count word
          if (rem < 4) return 1;
          if (p - base >= kWaveBlk) return 2;
          cnt = bswap32(__builtin_amdgcn_readfirstlane(blk[(p - base) >> 2]));
          p += 4;
          return 0;
        }
        ++pc;
        return kWalkCont;
      };
      do rc = OPS::visit(sops, pc, skel);
      while (rc == kWalkCont);
      if (!rc && (cnt > 1u || static_cast<uint64_t>(cnt) * emin > b - p)) rc = 1;
    }
    if (rc == 2) {  // the node leaves the block: write the batch, reload at the node
      if (!flush()) return false;
      if (base == (p0 & ~15ull)) return false;  // a node longer than the block
      p = p0;
      base = ~0ull;
      continue;
    }
    if (rc) return false;
    m_pc = lane == nb ? static_cast<uint32_t>(p0 - a) | cnt : m_pc;
    ++nb;
    ++k;
    if (!cnt) return finish(p);
    if (nb == 64u && !flush()) return false;
  }
}

template <class OPS>
__device__ __forceinline__ void sub_decode_kernel(XDRG_SUB_DECODE_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  load_ops(sops, ops, nops);
  // packed element areas (main pass): the wave's 64 records are one group
  uint64_t pk_cur = 0, pk_end = 0;
  if (P.packed && !P.list) {
    const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t r0 = r - (threadIdx.x & 63u);
    if (r0 < n) {  // wave-uniform
      const bool in = r < n;
      const uint64_t a = in ? offsets[r] : 0, b = in ? offsets[r + 1] : 0;
      const bool bad = in && (b < a || b > len);
      const bool on = in && !bad && a + mark <= b;
      const uint64_t e = on ? sub_ebytes(sops, table, xdr, a + mark, b) : 0u;
      const uint64_t E = on ? min(e, ebudget(F, a, b)) : 0u;
      (void)packed_area(E, bad, offsets[r0], ebase, F, pk_cur, pk_end);
    }
  }
  // the main pass's window (win_rd): [wb, wb + wl) of the stream, from the
  // wave's first record on
  uint64_t wb = 0;
  uint32_t wl = 0;
  const uint32_t *wbuf = nullptr;
  if (P.win && !P.list) {
    const uint64_t r0 = static_cast<uint64_t>(blockIdx.x) * blockDim.x + (threadIdx.x & ~63u);
    if (r0 < n) {  // wave-uniform
      const uint64_t a0 = offsets[r0], a1 = offsets[min(r0 + 64u, n)];
      wb = a0 & ~15ull;
      const uint64_t e = min(min(a1, len), wb + kWaveBlk);  // (offsets out of order: no window)
      wl = e > wb && a0 <= len ? static_cast<uint32_t>(e - wb) & ~3u : 0u;
      const uint32_t lo = (static_cast<uint32_t>(nops * sizeof(xdrg_op)) + 15u) & ~15u;
      uint32_t *buf = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(smem) + lo) +
                      (threadIdx.x / 64u) * (kWaveBlk / 4u);
      for (uint32_t k = threadIdx.x & 63u; 16u * k < wl; k += 64u) {
        const uint64_t o = wb + 16ull * k;
        u32x4 v{0u, 0u, 0u, 0u};
        if (16u * k + 16u <= wl) {
          v = ld16u(xdr + o);
        } else {
          v.x = ld32(xdr + o);
          if (16u * k + 8u <= wl) v.y = ld32(xdr + o + 4);
          if (16u * k + 12u <= wl) v.z = ld32(xdr + o + 8);
        }
        *reinterpret_cast<u32x4 *>(buf + 4u * k) = v;
      }
      wave_sync();
      wbuf = buf;
    }
  }
  sub_records<true>(P, n, [&](uint64_t r, auto &st) {
    const uint64_t a = offsets[r], b = offsets[r + 1];
    if (!P.list) {  // record-level checks: the main pass reports them once
      if (r == n - 1 && b != len) report(err, n, kOpRecordLevel, XDRG_ERR_TRAILING);
      if (b < a || b > len) { report(err, r, 0, XDRG_ERR_OVERFLOW_GET); return; }
      if (mark) {  // xdr_from_msg: the message read_message framed (srpc.cc:29-55)
        const uint32_t c = b - a < 4 ? XDRG_ERR_MSG_EOF : mark_code(ld32(xdr + a), b - a - 4);
        if (c) { report(err, r, kOpRecordLevel, c); return; }
      }
      if ((b - a) & 3u) { report(err, r, kOpRecordLevel, XDRG_ERR_SIZE_NOT_MULT4); return; }
      if (P.wave_list && b - a >= kWaveMin && !(a & 3u)) {  // the wave pass walks it
        P.wave_list[atomicAdd(P.wave_count, 1ull)] = static_cast<uint32_t>(r);
        return;
      }
    }
    uint32_t full_op = 0;
    const bool pk = P.packed && !P.list;
    const uint64_t e0 = pk ? pk_cur : ebase + static_cast<uint64_t>(F) * a;
    const uint64_t e1 = pk ? pk_end : ebase + static_cast<uint64_t>(F) * b;
    if constexpr (no_ref<decltype(st)>::kCap == kWaveFrames) {  // the wave pass
      {  // every value the wave's walk starts from, scalar
        const uint32_t lo = (static_cast<uint32_t>(nops * sizeof(xdrg_op)) + 15u) & ~15u;
        uint32_t *blk = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(smem) + lo) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x / 64u) * (kWaveBlk / 4u);
        const uint64_t ru = rfl64(r), au = rfl64(a), bu = rfl64(b);
        const uint32_t lvpc = list_vpc(sops, nops);
        uint16_t *nxt = P.win ? reinterpret_cast<uint16_t *>(reinterpret_cast<uint8_t *>(smem) + lo +
                                                             kWaveWaves * kWaveBlk) +
                                    __builtin_amdgcn_readfirstlane(threadIdx.x / 64u) * (kWaveBlk / 4u)
                              : nullptr;
        if (lvpc != ~0u && list_decode<OPS>(sops, lvpc, table, xdr, au + mark, bu, native + ru * stride, stride,
                                            heap, ebase + static_cast<uint64_t>(F) * au,
                                            ebase + static_cast<uint64_t>(F) * bu, stack_limit, blk, nxt))
          return;
        if (sub_decode_rec<OPS>(sops, table, xdr, au + mark, bu, native + ru * stride, stride, heap,
                                ebase + static_cast<uint64_t>(F) * au, ebase + static_cast<uint64_t>(F) * bu,
                                stack_limit, ru, err, &full_op, st, true, wave_rd{xdr, bu, blk, ~0ull}) == kWalkFull &&
            !(threadIdx.x & 63u))  // (one lane lists it)
          sub_full(P, ru, full_op, XDRG_ERR_STACK_GET, err);
      }
    } else {
      int rc;
      if constexpr (no_ref<decltype(st)>::kCap == kSubFrames)  // main pass
        rc = sub_decode_rec<OPS>(sops, table, xdr, a + mark, b, native + r * stride, stride, heap, e0, e1,
                                 stack_limit, r, err, &full_op, st, P.defer != nullptr,
                                 win_rd{xdr, wbuf, wb, (a & 3u) ? 0u : wl});
      else
        rc = sub_decode_rec<OPS>(sops, table, xdr, a + mark, b, native + r * stride, stride, heap, e0, e1,
                                 stack_limit, r, err, &full_op, st, P.defer != nullptr, glob_rd{xdr});
      if (rc == kWalkFull) sub_full(P, r, full_op, XDRG_ERR_STACK_GET, err);
    }
  });
}

}  // namespace dev
}  // namespace xdrg
