/*
 * xdrgpu.h — C ABI of the MI355X-native batched XDR (RFC 4506) marshal engine.
 *
 * This is the drop-in boundary for xdrpp's encode/decode hot path.  Every
 * entry point below replaces one reference interface; the reference
 * file:line it stands in for is cited next to it (paths relative to the
 * xdrpp source tree):
 *
 *   xdrg_plan_create      <- the compile-time field walk xdr_traits<T>::save/load
 *                            performs (xdrc/gen_hh.cc:212-250 structs,
 *                            :575-675 unions; xdrpp/types.h:676-730)
 *   xdrg_encode           <- xdr_to_opaque(r0, ..., rN-1)   xdrpp/marshal.h:264-272
 *                            (xdr_generic_put, xdrpp/marshal.h:84-137)
 *   xdrg_encode_sizes /   <- its two halves: xdr_argpack_size, then the put
 *   xdrg_encode_sized        xdrpp/marshal.h:223-234, :264-272
 *   xdrg_decode           <- xdr_from_opaque(bytes, r...)    xdrpp/marshal.h:299-306
 *                            (xdr_generic_get, xdrpp/marshal.h:142-211)
 *   xdrg_encode_msgs      <- xdr_to_msg(r) per record       xdrpp/marshal.h:252-260
 *                            (record mark: message_t::alloc, xdrpp/marshal.cc:15-31)
 *   xdrg_decode_msgs      <- xdr_from_msg(m, r) per message  xdrpp/marshal.h:278-284
 *   xdrg_index_records    <- the record boundaries of xdr_from_opaque's walk
 *                                                            xdrpp/marshal.h:299-306
 *   xdrg_index_msgs       <- the record-mark framing of read_message /
 *                            msg_sock::input                 xdrpp/srpc.cc:29-55,
 *                                                            xdrpp/msgsock.cc:38-119
 *   xdrg_serial_sizes     <- xdr_argpack_size / xdr_size     xdrpp/marshal.h:223-234,
 *                                                            xdrpp/types.h:240-244
 *   xdrg_record_depths    <- check_xdr_depth / depth_checker xdrpp/depth_checker.h:10-79
 *   xdrg_swap32/xdrg_swap64 <- swap32 / swap64               xdrpp/endian.h:56-68
 *   xdrg_rpc_dispatch     <- rpc_server_base::dispatch header decode + routing
 *                            xdrpp/server.cc:78-117, srpc.h:121-128
 *   xdrg_rpc_check_replies <- check_call_hdr + xid test      xdrpp/rpc_msg.cc:115-131,
 *                                                            xdrpp/srpc.h:61-66
 *   xdrg_rpc_replies      <- rpc_*_msg error replies         xdrpp/server.cc:8-67
 *   xdrg_error_message    <- the what() strings of the exception types
 *                            xdrpp/types.h:57-99, marshal.h:104-108,152-170,
 *                            :131-136,:207-210, marshal.cc:43-57
 *
 * Conventions
 *  - All data pointers passed to encode/decode are DEVICE pointers
 *    (hipMalloc / torch CUDA tensors).  No allocation happens inside the
 *    encode/decode calls; scratch comes from a caller-provided workspace.
 *  - Calls are stream-ordered and asynchronous.  Errors found by the
 *    kernels are recorded in a device-resident xdrg_status that the caller
 *    reads back with xdrg_status_read (which synchronises the stream).
 *  - No C++ exceptions cross this boundary.  Return values are
 *    XDRG_OK or a negative XDRG_E* API error; data errors are positive
 *    XDRG_ERR_* codes reported through xdrg_status.
 *  - "Native" records are the in-memory representation the kernels read
 *    (encode) or write (decode): for fixed-size schemas this is exactly the
 *    C++ struct produced by xdrc; variable-length bytes fields are staged as
 *    an xdrg_bytes_ref into a byte heap (std::vector / std::string storage is
 *    not device addressable).  See DESIGN.md "Data layout in HBM".
 */
#ifndef XDRGPU_H_INCLUDED
#define XDRGPU_H_INCLUDED 1

#ifdef __HIPCC_RTC__ /* plan-specialized kernels compiled by hiprtc */
#include <stdint.h>
#else
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define XDRG_ABI_VERSION 8  /* 8: XDRG_SUB_FRAMES 32 -> 8 (register frames) */

/* ---------------------------------------------------------------------- */
/* Plan ops: a flat, wire-ordered walk of xdr_traits<T>::save.             */
/* ---------------------------------------------------------------------- */

enum xdrg_op_kind {
  XDRG_OP_U32 = 1,       /* int / unsigned / float: 4-byte native, 4-byte wire   (types.h:286-332) */
  XDRG_OP_U64 = 2,       /* hyper / unsigned hyper / double                     (types.h:286-332) */
  XDRG_OP_BOOL = 3,      /* 1-byte native bool, wire u32 0/1; any nonzero decodes true (types.h:335-349) */
  XDRG_OP_ENUM = 4,      /* int32 native; arg0/arg1 = enum value list in table (gen_hh.cc:271-305) */
  XDRG_OP_OPAQUE = 5,    /* opaque[arg0]: fixed bytes, wire pad4(arg0)          (types.h:455-470) */
  XDRG_OP_VAROPAQUE = 6, /* opaque<arg0>: native xdrg_bytes_ref                 (types.h:515-524) */
  XDRG_OP_STRING = 7,    /* string<arg0>: native xdrg_bytes_ref                 (types.h:530-587) */
  XDRG_OP_UNION = 8,     /* discriminant int32 at noff, then the selected arm   (gen_hh.cc:639-673) */
  XDRG_OP_JUMP = 9,      /* pc = arg0 (end of a union arm)                      */
  XDRG_OP_END = 10,      /* end of record                                       */
  XDRG_OP_VECTOR = 11    /* xvector<T,arg0> / pointer<T> (F_POINTER, arg0 = 1):  (types.h:365-414,476-512,591-665)
                          * native xdrg_bytes_ref {heap offset, count} of an
                          * element array with stride arg1; wire u32 count then
                          * the elements.  Fixed-size elements: the element's
                          * ops follow inline, ops [pc+1, pc+1+arg2).  Any
                          * element (F_SUB): the element is a subroutine, ops
                          * from pc arg4 to the next END, walked once per
                          * element (arg2 = 0); it may be the plan's own
                          * record (recursive types). */
};

enum xdrg_op_flags {
  XDRG_F_VALIDATE = 1,   /* ENUM / UNION: opt-in xdr_validate_enum (types.h:157-173) */
  XDRG_F_DEFAULT = 2,    /* UNION: has a default arm; arg4 = its pc             */
  XDRG_F_POINTER = 4,    /* VECTOR: xdr::pointer (count 0 or 1)                 */
  XDRG_F_SUB = 8         /* VECTOR: element subroutine at pc arg4 (below)       */
};

/*
 * One plan op (32 bytes).  `depth` is the number of class/container levels
 * (xdr_generic_put/get operator() for is_class||is_container,
 * marshal.h:129-136 and :198-205) enclosing the op, the top-level record
 * counting as 1; a union op counts its own level.  The kernels raise the
 * stack-overflow error when depth > stack_limit, which is what
 * marshaling_stack_limit (marshal.h:21,34) does in the reference.
 *
 *   kind       arg0              arg1          arg2             arg3     arg4
 *   U32/U64/BOOL  -              -             -                -        -
 *   ENUM       table idx         count         -                -        -
 *   OPAQUE     length            -             -                -        -
 *   VAROPAQUE  max length        -             -                -        -
 *   STRING     max length        -             -                -        -
 *   UNION      enum table idx    enum count    case table idx   ncases   default pc
 *   JUMP       target pc         -             -                -        -
 *
 *   VECTOR     max count         elem stride   inline ops       -        F_SUB: body pc
 *
 * The case table is a run of (int32 value, uint32 target pc) pairs in the
 * shared uint32 table.  `name` is an opaque caller id (for messages).
 *
 * Element subroutines (F_SUB).  The record's ops end with END; subroutine
 * bodies follow it, each ending with its own END.  A body's field offsets
 * are relative to the element and its depths relative to the VECTOR op:
 * an op of a body entered from a VECTOR op at (absolute) depth d sits at
 * depth d + op.depth, so an element struct's fields are at d + 1 exactly
 * as if the element were written inline.  A body may be entered from
 * itself (test_recursive, tests/xdrtest.x:29-33; rpcbind's rp__list,
 * xdrpp/rpcb_prot.x:34).  Nesting is bounded by the data and by
 * marshaling_stack_limit only: a walk keeps XDRG_SUB_FRAMES element frames
 * in registers, and records nested deeper are walked again by deep passes
 * whose frames live in the caller's workspace
 * (xdrg_deep_workspace_size: about 218 MiB + 12 bytes per record for a plan
 * that can nest that deep, 0 for any other).  A record that needs more than XDRG_MAX_FRAMES nested element
 * frames raises the stack-overflow error at the VECTOR op that would open
 * the next one; the reference's own recursion ends far earlier, in a
 * segmentation fault of its 8 MiB call stack.  A decode that fails inside
 * elements leaves rsv = 1 + the failing element's index in every container
 * on the way to the failure (0 in the others).
 */
#define XDRG_SUB_FRAMES 8
/* Element frames the record index's parse follows (xdrg_index_records);
 * a record nested deeper is XDRG_ERR_INDEX_LONG, as one past the window. */
#define XDRG_INDEX_FRAMES 16
#define XDRG_MAX_FRAMES (1u << 19)
typedef struct xdrg_op {
  uint8_t kind;
  uint8_t flags;
  uint16_t depth;
  uint32_t noff; /* byte offset of the field in the native record */
  uint32_t arg0;
  uint32_t arg1;
  uint32_t arg2;
  uint32_t arg3;
  uint32_t arg4;
  uint32_t name;
} xdrg_op;

/* Staged representation of a variable-length opaque<>/string<> field. */
typedef struct xdrg_bytes_ref {
  uint64_t off; /* byte offset into the heap buffer */
  uint32_t len; /* number of payload bytes          */
  uint32_t rsv; /* must be zero                      */
} xdrg_bytes_ref;

typedef struct xdrg_plan xdrg_plan;

enum xdrg_path {
  XDRG_PATH_FIXED_REG = 1, /* fixed size, identity layout: register permute kernel */
  XDRG_PATH_FIXED_LDS = 2, /* fixed size, general layout: LDS-staged gather kernel */
  XDRG_PATH_VAR = 3        /* variable length / unions: size pass + scan + interpreter */
};

typedef struct xdrg_plan_info {
  uint32_t path;          /* enum xdrg_path */
  uint32_t native_stride; /* bytes per native record */
  uint32_t fixed_size;    /* wire bytes per record if fixed, else 0 */
  uint32_t max_depth;     /* deepest op depth */
  uint32_t nops;
  uint32_t has_checks;    /* decode validates something (pads, enums) */
  uint64_t max_record_bytes; /* largest wire record the plan's bounds allow
                              * (fixed: fixed_size); a message's body bound */
  uint32_t group_records;    /* FIXED_LDS plans run by the group kernel: records
                              * per group (0: the LDS kernel, or not fixed) */
  uint32_t specialized;      /* var plans: 1 when the plan's specialized kernels
                              * are built (xdrg_plan_build_kernels) */
} xdrg_plan_info;

/* ---------------------------------------------------------------------- */
/* Status / errors                                                         */
/* ---------------------------------------------------------------------- */

/* API errors (return values). */
#define XDRG_OK 0
#define XDRG_EINVAL (-1)
#define XDRG_EALIGN (-2)
#define XDRG_EUNSUPPORTED (-3)
#define XDRG_EHIP (-4)
#define XDRG_ENOMEM (-5)
#define XDRG_ESPACE (-6) /* workspace or output buffer too small */

/* Data errors (reported through xdrg_status); each maps to one reference
 * exception class and what() string, see xdrg_error_message. */
enum xdrg_err {
  XDRG_ERR_NONE = 0,
  XDRG_ERR_OVERFLOW_GET = 1,    /* xdr_overflow        marshal.h:166-170 */
  XDRG_ERR_OVERFLOW_PUT = 2,    /* xdr_overflow        marshal.h:104-108 */
  XDRG_ERR_XVECTOR_BOUND = 3,   /* xdr_overflow        types.h:486-489   */
  XDRG_ERR_XSTRING_BOUND = 4,   /* xdr_overflow        types.h:539-542   */
  XDRG_ERR_NONZERO_PAD = 5,     /* xdr_should_be_zero  marshal.cc:52-55  */
  XDRG_ERR_BAD_DISCRIMINANT = 6,/* xdr_bad_discriminant gen_hh.cc:479-481,645,658 */
  XDRG_ERR_INVALID_ENUM = 7,    /* xdr_invariant_failed types.h:168-170  */
  XDRG_ERR_STACK_PUT = 8,       /* xdr_stack_overflow  marshal.h:131-132 */
  XDRG_ERR_STACK_GET = 9,       /* xdr_stack_overflow  marshal.h:200-201 */
  XDRG_ERR_SIZE_NOT_MULT4 = 10, /* xdr_bad_message_size marshal.h:157-159 */
  XDRG_ERR_TRAILING = 11,       /* xdr_bad_message_size marshal.h:207-210 */
  XDRG_ERR_POINTER_BOUND = 12,  /* xdr_overflow        types.h:605-608   */
  /* Record-marked message framing (RFC 5531 record marks of message_t). */
  XDRG_ERR_MSG_EOF = 13,        /* xdr_bad_message_size srpc.cc:36-37,51-52 */
  XDRG_ERR_MSG_SIZE4 = 14,      /* xdr_bad_message_size srpc.cc:38-39    */
  XDRG_ERR_MSG_FRAGMENT = 15,   /* xdr_bad_message_size srpc.cc:42-45    */
  XDRG_ERR_MSG_TOO_LONG = 16,   /* msg_sock maxmsglen_  msgsock.cc:99-111 */
  XDRG_ERR_MSG_MISMATCH = 17,   /* mark disagrees with the record index  */
  XDRG_ERR_MSG_COUNT = 18,      /* more messages than the index can hold */
  XDRG_ERR_LOOKBACK = 19,      /* internal: a block of the one-pass encode waited
                                   too long for the byte total of the blocks before
                                   it (never expected; the output is not written) */
  XDRG_ERR_INDEX_LONG = 20      /* xdrg_index_records: a record longer than its bound */
};

/* Exception class a data error maps to (for host-side rethrow). */
enum xdrg_exc {
  XDRG_EXC_NONE = 0,
  XDRG_EXC_OVERFLOW = 1,          /* xdr::xdr_overflow */
  XDRG_EXC_STACK_OVERFLOW = 2,    /* xdr::xdr_stack_overflow */
  XDRG_EXC_BAD_MESSAGE_SIZE = 3,  /* xdr::xdr_bad_message_size */
  XDRG_EXC_BAD_DISCRIMINANT = 4,  /* xdr::xdr_bad_discriminant */
  XDRG_EXC_SHOULD_BE_ZERO = 5,    /* xdr::xdr_should_be_zero */
  XDRG_EXC_INVARIANT_FAILED = 6   /* xdr::xdr_invariant_failed */
};

/*
 * Device-resident status block.  first_error packs the lowest failing
 * (record, op) pair: (record << 24) | (op << 8) | code; all-ones = no error.
 * The lowest record wins because the reference stops at the first failing
 * record of the concatenated stream; within a record the lowest op index
 * wins because the reference walks fields in wire order.
 */
typedef struct xdrg_status {
  uint64_t first_error;
  uint64_t total_bytes; /* var encode: total wire bytes produced */
} xdrg_status;

typedef struct xdrg_error {
  int32_t code;     /* enum xdrg_err */
  int32_t exc;      /* enum xdrg_exc */
  uint64_t record;  /* index of the failing record */
  uint32_t op;      /* plan op index within the record (0xffffffff: record level) */
  uint32_t rsv;
  uint64_t total_bytes;
} xdrg_error;

/* ---------------------------------------------------------------------- */
/* Entry points                                                            */
/* ---------------------------------------------------------------------- */

int xdrg_abi_version(void);

/*
 * Graph capture.  Every encode, decode, size, depth, message and RPC call
 * can be captured into a hipGraph (stream capture) and replayed any number
 * of times, except xdrg_index_records' default wait for its walk's verdict
 * (a capturing stream stays asynchronous instead) and xdrg_index_msgs past
 * 16,380-byte messages.  The captured graph holds kernels only: the
 * library fills and copies device memory with kernels of its own, because
 * memset nodes of 16 bytes or more do not take effect on the replays after
 * the first under ROCm's graph packet capture (DEBUG_CLR_GRAPH_PACKET_
 * CAPTURE, on by default; tools/gpu/graph_node_probe.py, profiles/r05e),
 * which left the deep passes' list counters stale and faulted a recursive
 * plan's second replay (profiles/r04c, r05a-d).  Kernels with private
 * (scratch) memory replay correctly, also when the runtime grows its
 * scratch area between replays (profiles/r06_graph): the two interpreter
 * kernels that keep private memory (the window decode of a plan run without
 * its specialized kernels, and the encode interpreter at
 * XDRG_OPT_ENC_UNROLL 16) are capturable like the rest.  Run a plan's first
 * launch on a device outside the capture (it uploads the plan's tables).
 */

/* Validate and compile an immutable plan.  `table` holds enum value lists
 * and union case tables referenced by the ops.  native_stride is the byte
 * distance between consecutive native records.  Host-only: the plan's
 * device tables are uploaded (synchronously) to each device by its first
 * launch on that device, so run one launch per device before capturing a
 * plan's launches into a hipGraph.  A plan of 65535 or more ops is
 * XDRG_EUNSUPPORTED (status keys hold a 16-bit op index). */
int xdrg_plan_create(const xdrg_op *ops, uint32_t nops, const uint32_t *table,
                     uint32_t ntable, uint32_t native_stride, xdrg_plan **out);
void xdrg_plan_destroy(xdrg_plan *plan);
int xdrg_plan_get_info(const xdrg_plan *plan, xdrg_plan_info *info);

/* Launch options of one plan (no reference counterpart: kernel choices and
 * launch shapes, for tests and tuning).  Every option defaults to the
 * automatic choice.  Options belong to the plan, not to the process; set
 * them before the plan is shared between threads.  Returns XDRG_EINVAL for
 * an unknown option or value. */
enum xdrg_plan_option {
  XDRG_OPT_VAR_ENCODE_KERNEL = 1, /* 0 auto, 1 per-lane walk, 3 chunk-map image   */
  XDRG_OPT_VAR_DECODE_KERNEL = 2, /* 0 auto, 1 per-lane walk, 2 LDS window         */
  XDRG_OPT_FIXED_PATH = 3,        /* non-identity layouts: 0 auto (tile kernel),
                                     2 LDS term kernel, 3 group kernel            */
  XDRG_OPT_IMAGE_BYTES = 4,       /* var encode LDS image per wave, -1 auto        */
  XDRG_OPT_WINDOW_BYTES = 5,      /* var decode LDS window per wave, -1 auto       */
  XDRG_OPT_ENC_UNROLL = 6,        /* payload chunks in flight per lane: 4, 8, 16   */
  XDRG_OPT_DEC_READAHEAD = 7,     /* window decode 32-byte read-ahead: 0 / 1       */
  XDRG_OPT_SIZE_LINEAR = 8,       /* walk-free size pass for linear plans: 0 / 1;
                                     -1 (default) only without generated kernels */
  XDRG_OPT_GRP_UNROLL = 9,        /* fixed group kernel chunks in flight, 0 auto   */
  XDRG_OPT_GRP_BLOCKS = 10,       /* fixed group kernel workgroups, 0 auto         */
  XDRG_OPT_GRP_NONTEMPORAL = 11,  /* fixed group kernel non-temporal stores: 0 / 1 */
  XDRG_OPT_SPECIALIZE = 12,       /* var plans: 1 (default) run the plan-specialized
                                     kernels (built by the first launch, or
                                     xdrg_plan_build_kernels); 0 the interpreter */
  XDRG_OPT_STAGE_BYTES = 14,     /* window decode, plans with fixed-element
                                     containers: LDS stage of a 64-record group's
                                     element arrays (written out as whole lines
                                     after the walk), -1 auto, 0 none           */
  XDRG_OPT_ENC_STREAM = 15,      /* plan-specialized word-list plans: -1 (default)
                                     the size pass + scan + a record kernel that
                                     walks each record once, first; 1 the same
                                     record kernel with no size pass and no scan
                                     (xdrg_encode: each wave's base by a look-back
                                     over the byte totals of the waves before it);
                                     0 the record kernel that walks per window   */
  XDRG_OPT_FIXED_STREAM = 16,    /* identity fixed plans (k_fixed_reg) launch
                                     shape: -1 (default) by working set (in+out
                                     past 384 MiB: non-temporal one-shot grid,
                                     else plain 1024 workgroups); 0 plain 1024;
                                     1 non-temporal one-shot; 2 plain one-shot;
                                     3 non-temporal 1024                         */
  XDRG_OPT_INDEX_FAST = 13        /* xdrg_index_records: 1 (default) the speculative
                                     chain walk first, then the call waits for its
                                     verdict and runs the list ranking only when a
                                     check failed; 2 the same without the wait (the
                                     list ranking is queued and skips itself: the
                                     call stays asynchronous); 0 the list ranking
                                     alone.  Same offsets, count and errors.
                                     3 (a tuning aid) the walk alone, waited for:
                                     when a check fails nothing else runs, the
                                     offsets are left as they were and the
                                     workspace keeps the walk's segment records */
};
int xdrg_plan_set_option(xdrg_plan *plan, int option, int64_t value);

/* ---------------------------------------------------------------------- */
/* Plan-specialized kernels (var plans)                                    */
/* ---------------------------------------------------------------------- */
/*
 * The generation-time form of xdr_traits<T>::save/load (xdrc/gen_hh.cc:
 * 212-250, :575-675): a plan's walk emitted as straight-line HIP source --
 * every field's checks, swaps and bytes, unions as switch statements,
 * containers as loops -- over the library's var kernels, compiled for
 * gfx950; also the plan's record-start parse for xdrg_index_records.  No
 * reference interface corresponds one to one: this is the back end xdrc
 * would run beside gen_hh.
 *
 *   xdrg_plan_kernel_source  the plan's source (NUL-terminated into buf when
 *                            cap > 0; *len = its length).  XDRG_EUNSUPPORTED
 *                            for fixed plans (their kernels are generic).
 *   xdrg_plan_build_kernels  compile now: from the kernel cache (files named
 *                            by a hash of the source under $XDRG_KERNEL_CACHE,
 *                            default kernel_cache/ beside libxdrgpu.so) or
 *                            with hiprtc.  The first var launch does this on
 *                            its own; XDRG_EHIP carries the compile log.
 *   xdrg_plan_load_kernels   attach a code object compiled ahead of time
 *                            from xdrg_plan_kernel_source (before the plan's
 *                            first launch).
 */
int xdrg_plan_kernel_source(const xdrg_plan *plan, char *buf, size_t cap, size_t *len);
int xdrg_plan_build_kernels(xdrg_plan *plan);
int xdrg_plan_load_kernels(xdrg_plan *plan, const void *code_object, size_t size);

/* Workspace bytes encode (var plans) and encode_msgs (any plan) need for n
 * records; it includes xdrg_deep_workspace_size. */
size_t xdrg_workspace_size(const xdrg_plan *plan, uint64_t n);
/* Workspace bytes decode, decode_msgs, serial_sizes and record_depths need
 * for n records: 0 except for plans whose element subroutines can nest past
 * XDRG_SUB_FRAMES, whose deep passes keep their lists of deferred records
 * and their frame slabs there, and the size walk its log of long chains
 * (about 218 MiB + 12 bytes per record; 256-byte aligned).  The memory is the caller's: no call allocates, locks or keeps
 * state between calls, so calls on different streams with different
 * workspaces run side by side, and a captured graph of them holds kernels
 * only (see "Graph capture" below). */
size_t xdrg_deep_workspace_size(const xdrg_plan *plan, uint64_t n);

/* Zero a status block (first_error = all ones) on `stream`. */
int xdrg_status_init(xdrg_status *d_status, void *stream);
/* Synchronise `stream`, then read and decode the status block. */
int xdrg_status_read(const xdrg_status *d_status, void *stream, xdrg_error *out);

/*
 * Encode n native records to the concatenated XDR stream, i.e. the bytes of
 * xdr_to_opaque(r0, ..., rn-1).
 *   d_native    n records, native_stride apart
 *   d_heap      byte heap the xdrg_bytes_ref fields point into (var plans)
 *   heap_len    heap size in bytes (reads are clamped to it)
 *   d_xdr       output; xdr_capacity bytes available
 *   d_offsets   var plans: out, n+1 uint64 record offsets (record i occupies
 *               [off[i], off[i+1]); off[n] = total).  May be NULL for fixed.
 *   stack_limit marshaling_stack_limit in effect (0xffffffff = default)
 * For a fixed plan the output is exactly n * fixed_size bytes.
 */
int xdrg_encode(const xdrg_plan *plan, const void *d_native, uint64_t n,
                const uint8_t *d_heap, uint64_t heap_len, void *d_xdr,
                uint64_t xdr_capacity, uint64_t *d_offsets,
                uint32_t stack_limit, void *d_workspace, size_t workspace_bytes,
                xdrg_status *d_status, void *stream);

/*
 * xdrg_encode (msgs = 0) or xdrg_encode_msgs (msgs = 1) in two halves, for
 * callers that size the output from the records, as xdr_to_opaque does
 * (xdr_argpack_size, then xdr_generic_put; xdrpp/marshal.h:264-272):
 *   xdrg_encode_sizes  the size pass alone (xdr_size of every record, their
 *                      scan into the workspace); the total wire bytes land
 *                      in d_status->total_bytes and size errors (a bad
 *                      discriminant) in d_status.  No output is written.
 *   xdrg_encode_sized  the encode over the sizes the first half left in the
 *                      same workspace, with the same status block (not
 *                      re-initialised), records, heap and msgs flag: the
 *                      size pass does not run again (plans whose element
 *                      subroutines nest past XDRG_SUB_FRAMES: the encode's
 *                      deep passes walk the lists of deferred records the
 *                      size pass left in the workspace).
 * Arguments as xdrg_encode / xdrg_encode_msgs; d_offsets is required by the
 * second half for every plan with msgs, for var plans without.
 */
int xdrg_encode_sizes(const xdrg_plan *plan, const void *d_native, uint64_t n,
                      const uint8_t *d_heap, uint64_t heap_len, uint32_t stack_limit, int msgs,
                      void *d_workspace, size_t workspace_bytes, xdrg_status *d_status, void *stream);
int xdrg_encode_sized(const xdrg_plan *plan, const void *d_native, uint64_t n,
                      const uint8_t *d_heap, uint64_t heap_len, void *d_out, uint64_t out_capacity,
                      uint64_t *d_offsets, uint32_t stack_limit, int msgs, void *d_workspace,
                      size_t workspace_bytes, xdrg_status *d_status, void *stream);

/*
 * Decode n records from an XDR stream of xdr_len bytes.
 * Fixed plans: the stream is n * fixed_size bytes (the records' offsets are
 *   implied); a shorter stream fails the record it runs out in
 *   (xdr_overflow), a longer one fails with "did not consume whole message",
 *   exactly as xdr_from_opaque(bytes, r0, ..., rn-1) would.
 * Var plans: d_offsets (n+1 entries, from the encoder or from RPC record
 *   framing) is required; record i is decoded from [off[i], off[i+1]) with
 *   the semantics of xdr_from_opaque on that slice.  The decoded heap is
 *   the stream itself: d_heap_out (at least xdr_len bytes) receives the
 *   stream bytes verbatim, and every decoded xdrg_bytes_ref holds the stream
 *   offset of its payload (so payloads are never gathered one by one).
 *   Passing d_heap_out == d_xdr decodes without copying: the refs then
 *   point into the input stream, which must outlive the decoded records.
 * Workspace: xdrg_deep_workspace_size(plan, n) bytes (NULL/0 for plans
 * that need none).
 */
int xdrg_decode(const xdrg_plan *plan, const void *d_xdr, uint64_t xdr_len,
                const uint64_t *d_offsets, uint64_t n, void *d_native,
                uint8_t *d_heap_out, uint64_t heap_capacity,
                uint32_t stack_limit, void *d_workspace, size_t workspace_bytes,
                xdrg_status *d_status, void *stream);

/* Heap capacity xdrg_decode needs for a stream of xdr_len bytes: xdr_len,
 * plus, for plans with xvector<T>/pointer<T> fields, an area for the
 * decoded element arrays, F * xdr_len bytes from byte align16(xdr_len),
 * every array 8-byte aligned.  F = 1 + the largest native/wire size ratio
 * of an element type.  Plans whose containers all hold fixed-size elements
 * pack the arrays of each group of 64 records (records 64g .. 64g+63) back
 * to back from align8(align16(xdr_len) + F * off[64g]), record by record
 * (a record's share is what its counts ask for, each array rounded up to
 * 8 bytes), so the arrays leave as whole cache lines; F carries 2 more for
 * that rounding.  Plans with element subroutines place record i's arrays
 * from align16(xdr_len) + F * off[i] (F: the subroutine bound, + 2).  Only
 * the xdrg_bytes_ref offsets say where an array is. */
uint64_t xdrg_decode_heap_size(const xdrg_plan *plan, uint64_t xdr_len);

/* ---------------------------------------------------------------------- */
/* Record-marked batches: message_t buffers (RFC 5531 record marking)      */
/* ---------------------------------------------------------------------- */
/*
 * A message is a 4-byte record mark BE(size | 0x80000000) followed by
 * `size` bytes: message_t's raw_data()/raw_size() (xdrpp/message.h:33-64,
 * mark written by message_t::alloc, xdrpp/marshal.cc:15-31).  A batch is
 * messages back to back, which is what msg_sock::output writes for a queue
 * of messages (xdrpp/msgsock.cc:158-188) and what read_message /
 * msg_sock::input read (xdrpp/srpc.cc:29-55, msgsock.cc:38-119).
 */
#define XDRG_MARK_LAST 0x80000000u
/* Longest message one list-ranking window of the stream indexes holds (a
 * 16 KiB segment); xdrg_index_records' record bound. */
#define XDRG_INDEX_MAX_MSG 16380u
/* Longest message a record mark can state (31 size bits). */
#define XDRG_MAX_MSG 0x7fffffffu

/*
 * Encode n records as n messages: message i = xdr_to_msg(r_i)
 * (xdrpp/marshal.h:252-260).  Arguments as xdrg_encode; d_offsets is
 * required for every plan: d_offsets[i] = byte offset of message i's mark,
 * d_offsets[n] = total bytes.  The workspace is xdrg_workspace_size bytes.
 */
int xdrg_encode_msgs(const xdrg_plan *plan, const void *d_native, uint64_t n,
                     const uint8_t *d_heap, uint64_t heap_len, void *d_out,
                     uint64_t out_capacity, uint64_t *d_offsets, uint32_t stack_limit,
                     void *d_workspace, size_t workspace_bytes, xdrg_status *d_status,
                     void *stream);

/*
 * Decode n messages: message i occupies [d_offsets[i], d_offsets[i+1]) of
 * the stream (mark included) and decodes as xdr_from_msg(m_i, r_i)
 * (xdrpp/marshal.h:278-284).  The mark must be a last-fragment mark whose
 * size is the message's byte count (XDRG_ERR_MSG_* otherwise).  Heap
 * contract as xdrg_decode (refs are stream offsets); for plans without
 * opaque<>/string<>/xvector fields d_heap_out may be NULL.
 */
int xdrg_decode_msgs(const xdrg_plan *plan, const void *d_stream, uint64_t len,
                     const uint64_t *d_offsets, uint64_t n, void *d_native,
                     uint8_t *d_heap_out, uint64_t heap_capacity, uint32_t stack_limit,
                     void *d_workspace, size_t workspace_bytes, xdrg_status *d_status,
                     void *stream);

/*
 * Record index of a stream of messages, computed on the device: the
 * framing of read_message (srpc.cc:29-55) applied message after message,
 * plus msg_sock's length limit (maxmsglen_, msgsock.cc:99-111).  Writes
 * d_offsets[k] = byte offset of mark k for every message k, d_offsets[count]
 * = len, and *d_count (a device u64) = count.  On a framing error at
 * message k (premature EOF, fragment bit clear, size bits, too long, size
 * not a multiple of 4) the error is reported at record k through d_status,
 * *d_count = k and d_offsets[k] = the failing mark's offset.  At most
 * max_msgs messages are indexed (d_offsets holds max_msgs + 1 entries);
 * more is XDRG_ERR_MSG_COUNT at record max_msgs.  Entries past count are
 * unspecified.  Any max_msg_len up to XDRG_MAX_MSG: msg_sock's is 1 MiB by
 * default (msgsock.h:29), read_message has none.  Up to XDRG_INDEX_MAX_MSG
 * the marks are walked speculatively as for xdrg_index_records (the call
 * waits once for the walk's verdict, except on a stream being captured)
 * and a list-ranking pass runs when a check fails (a damaged stream, more
 * than max_msgs messages); past it the messages longer than that are
 * walked mark by mark on the device between list-ranking windows over the
 * rest, and the call waits on the stream once or twice per window (every
 * byte is read about twice at most).
 * Workspace: xdrg_index_workspace_size(len, max_msg_len).  Its contents are
 * the call's own: the path flag xdrg_index_records leaves in its last 256
 * bytes is not part of this call's contract (with max_msg_len past
 * XDRG_INDEX_MAX_MSG those bytes hold the windows' continuation block, and
 * the index pass's own 256-byte tail sits just before them).
 */
int xdrg_index_msgs(const void *d_stream, uint64_t len, uint32_t max_msg_len,
                    uint64_t max_msgs, uint64_t *d_offsets, uint64_t *d_count,
                    void *d_workspace, size_t workspace_bytes, xdrg_status *d_status,
                    void *stream);
size_t xdrg_index_workspace_size(uint64_t len, uint32_t max_msg_len);

/*
 * Record index of n records of `plan` concatenated in one stream, the
 * input of xdr_from_opaque(bytes, r0, ..., rn-1) (xdrpp/marshal.h:299-306),
 * computed on the device.  First a speculative walk: each 16 KiB segment
 * of the stream guesses where the chain of records enters it, walks the
 * chain (lengths, counts and discriminants only) and every guess is
 * checked against the previous segment's exit; when all hold and the chain
 * ends at len with exactly n records, that is the index.  Otherwise
 * (damaged streams, trailing or missing records, long records, or a guess
 * that missed: XDRG_OPT_INDEX_FAST = 0 forces this) every word position is
 * parsed as a possible record start and the chain of record ends from byte
 * 0 is ranked as for xdrg_index_msgs.  The first u32 of the 256 bytes
 * that end at xdrg_index_workspace_size(len, min(max_rec_len,
 * XDRG_INDEX_MAX_MSG)) -- the workspace's last 256 bytes when max_rec_len
 * <= XDRG_INDEX_MAX_MSG -- says which ran (1: the speculative walk).  By default
 * (XDRG_OPT_INDEX_FAST) the call waits on the stream once, for the walk's
 * verdict (not on a stream being captured into a graph: there it stays
 * asynchronous, as with XDRG_OPT_INDEX_FAST = 2).  Writes
 * d_offsets[0..n] for xdrg_decode: record r = [off[r], off[r+1]).  Where
 * the records stop parsing -- a bad discriminant, a length past its bound
 * or past the stream -- record k gets [off[k], len) and the rest [len, len),
 * so xdrg_decode reports the reference's error for record k; fewer than n
 * records end at len likewise, more leave off[n] < len (trailing bytes).
 * *d_count = the records the chain holds before it ends (all-ones when
 * it goes past record n).  max_rec_len <= XDRG_MAX_MSG.
 * max_rec_len <= XDRG_INDEX_MAX_MSG: a record longer than max_rec_len is
 * reported as XDRG_ERR_INDEX_LONG at its index.  Past XDRG_INDEX_MAX_MSG
 * the records have no length bound (xdr_from_opaque has none) and no
 * nesting bound but XDRG_MAX_FRAMES: with the plan's generated parse the
 * speculative walk takes the whole stream, records past its segments
 * parsed by a wave each through blocks of the stream in LDS (and a linked
 * list's plan, rpcb_prot.x's rp__list, parses its nodes in a loop); when
 * that walk misses the stream is indexed in rounds: one wave walks the
 * records longer than a window (lengths, counts and discriminants, its
 * element frames in the workspace) from where the chain stopped, then a
 * list-ranking window indexes the records after them up to the next long
 * one -- the call waits on the stream every round.  On a stream being
 * captured the walk runs alone, asynchronously: a stream it does not hold
 * gets the list ranking over records up to one window, which reports
 * XDRG_ERR_INDEX_LONG at a longer one (plans without the generated parse:
 * XDRG_EUNSUPPORTED).  Plans whose records can be empty are
 * XDRG_EUNSUPPORTED.  Workspace: xdrg_index_workspace_size(len,
 * max_rec_len).
 */
int xdrg_index_records(const xdrg_plan *plan, const void *d_xdr, uint64_t len, uint64_t n,
                       uint32_t max_rec_len, uint64_t *d_offsets, uint64_t *d_count,
                       void *d_workspace, size_t workspace_bytes, xdrg_status *d_status,
                       void *stream);

/* ---------------------------------------------------------------------- */
/* RPC header batches (RFC 5531 rpc_msg, xdrpp/rpc_msg.x)                  */
/* ---------------------------------------------------------------------- */
/*
 * A batch of record-marked messages (indexed by xdrg_index_msgs: message k
 * = [d_offsets[k], d_offsets[k+1]), mark first) has its rpc_msg headers
 * decoded, one lane per message, into xdrg_rpc_hdr records:
 *
 *   xdrg_rpc_dispatch      <- rpc_server_base::dispatch, header decode and
 *                             routing (xdrpp/server.cc:78-117) plus the
 *                             procedure lookup of srpc_service::process /
 *                             arpc_service::process (srpc.h:121-128,
 *                             arpc.h:175-182)
 *   xdrg_rpc_check_replies <- the client side: archive(g, hdr),
 *                             check_call_hdr (rpc_msg.cc:115-131) and the
 *                             xid test of synchronous_client_base::invoke
 *                             (srpc.h:61-66)
 *   xdrg_rpc_replies       <- rpc_accepted_error_msg, rpc_prog_mismatch_msg,
 *                             rpc_auth_error_msg, rpc_rpc_mismatch_msg
 *                             (server.cc:8-67): the error replies of a batch
 *                             as record-marked messages
 *
 * Success replies are xdr_to_msg(rpc_success_hdr(xid), res) (srpc.h:152,
 * server.h:27-49), i.e. an argument pack: encode them with xdrg_encode_msgs
 * and a plan whose record is {xid, REPLY, MSG_ACCEPTED, AUTH_NONE, 0,
 * SUCCESS, res...} (the Python/C++ layers build it).
 *
 * The header is decoded exactly as xdr_get decodes rpc_msg: a short message
 * is xdr_overflow, an opaque_auth body over 400 bytes is the xvector bound,
 * nonzero padding is xdr_should_be_zero, an unknown msg_type / reply_stat /
 * reject_stat is a bad discriminant (accept_stat has a default arm).  Enum
 * fields are not range-checked (no xdr_validate_enum in rpc_msg.x).  A
 * header that fails is not an error of the call: its record carries the
 * XDRG_ERR_* code in `err` and the action says what the reference does
 * with it (drop it, or raise in the client).
 */
enum xdrg_rpc_action {          /* server side (xdrg_rpc_dispatch)             */
  XDRG_RPC_DISPATCH = 0,        /* registered procedure: args at body_off     */
  XDRG_RPC_DROP_MALFORMED = 1,  /* header did not decode: dropped, no reply   server.cc:84-89 */
  XDRG_RPC_DROP_NONCALL = 2,    /* mtype != CALL: dropped, no reply           server.cc:90-93 */
  XDRG_RPC_RPC_MISMATCH = 3,    /* rpcvers != 2 -> rpc_rpc_mismatch_msg       server.cc:95-96 */
  XDRG_RPC_PROG_UNAVAIL = 4,    /* unknown prog                               server.cc:98-100 */
  XDRG_RPC_PROG_MISMATCH = 5,   /* unknown vers: low/high = registered range  server.cc:102-107 */
  XDRG_RPC_PROC_UNAVAIL = 6,    /* call_dispatch found no such proc           srpc.h:125-127 */
  XDRG_RPC_GARBAGE_ARGS = 7,    /* set by the caller when the args fail       srpc.h:132-134, server.cc:109-116 */
  XDRG_RPC_SYSTEM_ERR = 8,      /* set by the caller (accept_stat SYSTEM_ERR) */
  XDRG_RPC_AUTH_ERROR = 9       /* set by the caller: why in w[2]             server.cc:42-53 */
};
enum xdrg_rpc_status {          /* client side (xdrg_rpc_check_replies)        */
  XDRG_RPCR_OK = 0,             /* MSG_ACCEPTED + SUCCESS: result at body_off  */
  XDRG_RPCR_ACCEPT_STAT = 1,    /* xdr_call_error(accept_stat w[1])   rpc_msg.cc:120-122 */
  XDRG_RPCR_AUTH_STAT = 2,      /* xdr_call_error(auth_stat w[2])     rpc_msg.cc:124-125 */
  XDRG_RPCR_RPCVERS_MISMATCH = 3,/* xdr_call_error(RPCVERS_MISMATCH)  rpc_msg.cc:126 */
  XDRG_RPCR_NOT_REPLY = 4,      /* "call received when reply expected" rpc_msg.cc:117-118 */
  XDRG_RPCR_MALFORMED = 5,      /* archive(g, hdr) threw: code in err           srpc.h:62 */
  XDRG_RPCR_BAD_XID = 6         /* "synchronous_client: unexpected xid"         srpc.h:64-65 */
};
/* w[] slots of xdrg_rpc_hdr */
#define XDRG_RPC_W_RPCVERS 0     /* CALL  */
#define XDRG_RPC_W_PROG 1
#define XDRG_RPC_W_VERS 2
#define XDRG_RPC_W_PROC 3
#define XDRG_RPC_W_CRED_FLAVOR 4
#define XDRG_RPC_W_REPLY_STAT 0  /* REPLY */
#define XDRG_RPC_W_STAT 1        /*   accept_stat (MSG_ACCEPTED) or reject_stat (MSG_DENIED) */
#define XDRG_RPC_W_WHY 2         /*   auth_stat (AUTH_ERROR) */
#define XDRG_RPC_W_VERF_FLAVOR 5 /* both */
#define XDRG_RPC_W_LOW 6         /* PROG_MISMATCH / RPC_MISMATCH mismatch_info */
#define XDRG_RPC_W_HIGH 7

typedef struct xdrg_rpc_hdr {   /* 64 bytes */
  uint32_t xid;
  uint16_t action;   /* xdrg_rpc_action or xdrg_rpc_status */
  uint8_t err;       /* XDRG_ERR_* of a malformed header, else 0.  A malformed
                        header keeps only action, err, end and, for
                        XDRG_ERR_BAD_DISCRIMINANT, the union in w[0]
                        (0 _body_t, 1 reply_body, 2 rejected_reply) */
  uint8_t mtype;     /* msg_type as decoded */
  uint32_t w[8];     /* XDRG_RPC_W_* */
  uint32_t cred_len; /* CALL: cred body bytes (body at mark + 36) */
  uint32_t verf_len; /* verf body bytes (CALL: body ends at body_off; REPLY: at mark + 24) */
  uint64_t body_off; /* stream offset after the header: args (CALL) / results (REPLY) */
  uint64_t end;      /* stream offset of the message end */
} xdrg_rpc_hdr;

/* A registered procedure (prog, vers, proc).  The table passed to
 * xdrg_rpc_dispatch lists every procedure of every registered interface,
 * sorted by (prog, vers, proc), no duplicates: the servers_ map of
 * rpc_server_base (server.h:218-219) plus each interface's call_dispatch
 * switch (xdrc/gen_hh.cc:757-774). */
typedef struct xdrg_rpc_proc {
  uint32_t prog, vers, proc;
  uint32_t flags; /* 0, or XDRG_RPC_PROC_IFACE_ONLY: (prog, vers) is registered
                     but this entry names no procedure (an interface whose
                     call_dispatch has no case) */
} xdrg_rpc_proc;
#define XDRG_RPC_PROC_IFACE_ONLY 1u
#define XDRG_RPC_MAX_PROCS 4096u

int xdrg_rpc_dispatch(const void *d_stream, uint64_t len, const uint64_t *d_offsets,
                      uint64_t n, const xdrg_rpc_proc *d_procs, uint32_t nprocs,
                      xdrg_rpc_hdr *d_hdrs, void *stream);

/* d_xids: the xid each reply must carry (NULL: no xid test). */
int xdrg_rpc_check_replies(const void *d_stream, uint64_t len, const uint64_t *d_offsets,
                           uint64_t n, const uint32_t *d_xids, xdrg_rpc_hdr *d_hdrs,
                           void *stream);

/* Error replies of a dispatched batch, in message order: for every header
 * whose action is RPC_MISMATCH / PROG_UNAVAIL / PROG_MISMATCH /
 * PROC_UNAVAIL / GARBAGE_ARGS / SYSTEM_ERR / AUTH_ERROR one record-marked
 * message (28, 36 or 24 bytes with its mark); other actions add nothing.
 * d_offsets[i] = offset of header i's reply (== d_offsets[i+1] when it has
 * none), d_offsets[n] = total, also in d_status->total_bytes.  An output
 * capacity below the total is XDRG_ERR_OVERFLOW_PUT at the first reply that
 * does not fit.  Workspace: xdrg_rpc_replies_workspace_size(n) bytes. */
int xdrg_rpc_replies(const xdrg_rpc_hdr *d_hdrs, uint64_t n, void *d_out, uint64_t out_capacity,
                     uint64_t *d_offsets, void *d_workspace, size_t workspace_bytes,
                     xdrg_status *d_status, void *stream);
size_t xdrg_rpc_replies_workspace_size(uint64_t n);

/* Recursion depth per record: d_depths[i] = the deepest class/container
 * level record i's walk enters (the record itself is level 1), so
 * xdr::check_xdr_depth(r_i, limit) (xdrpp/depth_checker.h:72-79) is
 * d_depths[i] <= limit.  A bad union discriminant stops the walk and is
 * reported through d_status like the size pass.  d_heap: the staged heap
 * (element arrays of containers of variable-size elements are read from
 * it; NULL/0 when the plan has none). */
int xdrg_record_depths(const xdrg_plan *plan, const void *d_native, uint64_t n,
                       const void *d_heap, uint64_t heap_len, uint32_t *d_depths,
                       void *d_workspace, size_t workspace_bytes,
                       xdrg_status *d_status, void *stream);

/* Size pass alone: d_sizes[i] = xdr_size(record i) (uint32); d_heap as
 * for xdrg_record_depths.  Both take xdrg_deep_workspace_size(plan, n)
 * bytes of workspace (NULL/0 for every plan that needs none). */
int xdrg_serial_sizes(const xdrg_plan *plan, const void *d_native, uint64_t n,
                      const void *d_heap, uint64_t heap_len, uint32_t *d_sizes,
                      uint32_t stack_limit, void *d_workspace, size_t workspace_bytes,
                      xdrg_status *d_status, void *stream);

/* Bulk big-endian swaps (endian.h swap32/swap64) over device arrays. */
int xdrg_swap32(const uint32_t *d_in, uint32_t *d_out, uint64_t n, void *stream);
int xdrg_swap64(const uint64_t *d_in, uint64_t *d_out, uint64_t n, void *stream);

/* what() string and exception class of a data error.  For
 * XDRG_ERR_BAD_DISCRIMINANT the reference message names the union
 * ("bad value of <tag> in <union>"); the C++/Python layers format it from
 * the op's name id, this returns the generic prefix. */
const char *xdrg_error_message(int code);
int xdrg_error_exception(int code);

/* Last HIP error string recorded by this thread (for XDRG_EHIP). */
const char *xdrg_last_hip_error(void);

#ifdef __cplusplus
}
#endif

#endif /* XDRGPU_H_INCLUDED */
