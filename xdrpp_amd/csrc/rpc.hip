// RPC header batches on gfx950: rpc_msg header decode + routing of a batch
// of record-marked messages (the server's dispatch, the client's reply
// check) and the batch's error replies.  SURVEY.md §8 f1.
//
// Kernels
//   k_rpc_hdr<CLIENT>  one message per lane: decodes the rpc_msg header
//       exactly as xdr_get over xdr_traits<rpc_msg> does (xdrpp/rpc_msg.x,
//       xdrpp/marshal.h:142-211, marshal.cc:43-57) and routes it:
//       server  rpc_server_base::dispatch (xdrpp/server.cc:78-117) + the
//               procedure switch of srpc_service::process (srpc.h:121-128)
//               by binary search of a sorted (prog, vers, proc) table;
//       client  check_call_hdr (xdrpp/rpc_msg.cc:115-131) and the xid test
//               of synchronous_client_base::invoke (srpc.h:61-66).
//       A wave stages its 64 messages' stretch of the stream in LDS with
//       coalesced 16-byte loads and walks the headers from there; the
//       64-byte results leave through LDS as coalesced 16-byte stores.
//   k_rpc_reply_sizes / launch_block_scan / k_rpc_reply_emit  the error
//       replies (server.cc:8-67) as record-marked messages in message order:
//       per-256-header byte sums, the shared block scan, then each lane
//       writes its 0, 24, 28 or 36-byte message at its scanned offset.
#include <hip/hip_runtime.h>

#include "plan.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kMaxAuth = 400;  // opaque_auth body<400> (rpc_msg.x)

enum : uint32_t { CALL = 0, REPLY = 1 };
enum : uint32_t { MSG_ACCEPTED = 0, MSG_DENIED = 1 };
enum : uint32_t { SUCCESS = 0, PROG_UNAVAIL = 1, PROG_MISMATCH = 2, PROC_UNAVAIL = 3,
                  GARBAGE_ARGS = 4, SYSTEM_ERR = 5 };
enum : uint32_t { RPC_MISMATCH = 0, AUTH_ERROR = 1 };

__device__ __forceinline__ uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }
__device__ __forceinline__ uint32_t ld32(const uint8_t *s, uint64_t p) {
  return *reinterpret_cast<const uint32_t *>(s + p);
}

// -------------------------------------------------------- registry lookup
// Procedures sorted by (prog, vers, proc).  lower bound of the key on the
// first `level` fields (1: prog, 2: prog+vers, 3: all).
__device__ __forceinline__ bool key_less(const xdrg_rpc_proc &t, uint32_t P, uint32_t V,
                                         uint32_t Q, int level) {
  if (t.prog != P) return t.prog < P;
  if (level == 1) return false;
  if (t.vers != V) return t.vers < V;
  if (level == 2) return false;
  return t.proc < Q;
}
__device__ uint32_t lower(const xdrg_rpc_proc *t, uint32_t n, uint32_t P, uint32_t V, uint32_t Q,
                          int level) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (key_less(t[mid], P, V, Q, level)) lo = mid + 1; else hi = mid;
  }
  return lo;
}
// first entry with prog > P
__device__ uint32_t upper_prog(const xdrg_rpc_proc *t, uint32_t n, uint32_t P) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (t[mid].prog <= P) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// ------------------------------------------------------------ header walk
struct hdr_out {
  uint32_t xid = 0, action = 0, err = 0, mtype = 0;
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t cred_len = 0, verf_len = 0;
  uint64_t body_off = 0, end = 0;
};

// Payload cursor over [p, e) of the stream.  Words inside the wave's LDS
// window [wb, we) of the stream come from LDS, the rest from global memory.
struct cursor {
  const uint8_t *s;
  const uint32_t *win;
  uint64_t wb, we;
  uint64_t p, e;
  __device__ __forceinline__ uint32_t raw(uint64_t q) const {
    return q >= wb && q + 4 <= we ? win[(q - wb) >> 2] : ld32(s, q);
  }
  __device__ bool word(uint32_t &v) {  // xdr_generic_get::check(4) + get32
    if (e - p < 4) return false;
    v = bswap(raw(p));
    p += 4;
    return true;
  }
};

// opaque body<400> after its length word: check(size), resize (bound),
// get_bytes (pad check).  Returns 0 or an XDRG_ERR_* code.
__device__ uint32_t auth_body(cursor &c, uint32_t len) {
  if (len > c.e - c.p) return XDRG_ERR_OVERFLOW_GET;
  if (len > kMaxAuth) return XDRG_ERR_XVECTOR_BOUND;
  if (len & 3u) {
    const uint32_t w = c.raw(c.p + (len & ~3u));
    if (w & (0xffffffffu << (8u * (len & 3u)))) return XDRG_ERR_NONZERO_PAD;
  }
  c.p += (len + 3u) & ~3u;
  return 0;
}

// The header walk: 0 or an XDRG_ERR_* code; a bad discriminant carries
// the union in bits 8+ (0 _body_t, 1 reply_body, 2 rejected_reply).
// pre[] = the first eight payload words (independent
// loads issued together), nw = how many of them the message holds; the
// fixed-position prefix of a CALL (xid .. cred length) and of a REPLY
// (xid .. verf length) is read from them, the rest through the cursor.
__device__ uint32_t walk(cursor &c, const uint32_t (&pre)[8], uint32_t nw, hdr_out &h) {
  if (nw < 2) return XDRG_ERR_OVERFLOW_GET;
  h.xid = pre[0];
  h.mtype = pre[1];
  if (pre[1] == CALL) {
    // rpcvers, prog, vers, proc, cred.flavor, cred length
    if (nw < 8) return XDRG_ERR_OVERFLOW_GET;
    h.w[0] = pre[2]; h.w[1] = pre[3]; h.w[2] = pre[4]; h.w[3] = pre[5]; h.w[4] = pre[6];
    h.cred_len = pre[7];
    c.p += 32;
    uint32_t e = auth_body(c, h.cred_len);
    if (e) return e;
    if (!c.word(h.w[XDRG_RPC_W_VERF_FLAVOR])) return XDRG_ERR_OVERFLOW_GET;
    if (!c.word(h.verf_len)) return XDRG_ERR_OVERFLOW_GET;
    return auth_body(c, h.verf_len);
  }
  if (pre[1] != REPLY) return XDRG_ERR_BAD_DISCRIMINANT;  // site 0: _body_t
  if (nw < 3) return XDRG_ERR_OVERFLOW_GET;
  const uint32_t rs = pre[2];
  h.w[XDRG_RPC_W_REPLY_STAT] = rs;
  uint32_t v;
  if (rs == MSG_ACCEPTED) {
    if (nw < 5) return XDRG_ERR_OVERFLOW_GET;
    h.w[XDRG_RPC_W_VERF_FLAVOR] = pre[3];
    h.verf_len = pre[4];
    c.p += 20;
    uint32_t e = auth_body(c, h.verf_len);
    if (e) return e;
    if (!c.word(v)) return XDRG_ERR_OVERFLOW_GET;
    h.w[XDRG_RPC_W_STAT] = v;  // accept_stat: default arm is void
    if (v == PROG_MISMATCH) {
      if (!c.word(h.w[XDRG_RPC_W_LOW])) return XDRG_ERR_OVERFLOW_GET;
      if (!c.word(h.w[XDRG_RPC_W_HIGH])) return XDRG_ERR_OVERFLOW_GET;
    }
    return 0;
  }
  if (rs != MSG_DENIED) return XDRG_ERR_BAD_DISCRIMINANT | (1u << 8);  // reply_body
  if (nw < 4) return XDRG_ERR_OVERFLOW_GET;
  v = pre[3];
  h.w[XDRG_RPC_W_STAT] = v;
  if (v == RPC_MISMATCH) {
    if (nw < 6) return XDRG_ERR_OVERFLOW_GET;
    h.w[XDRG_RPC_W_LOW] = pre[4];
    h.w[XDRG_RPC_W_HIGH] = pre[5];
    c.p += 24;
    return 0;
  }
  if (v != AUTH_ERROR) return XDRG_ERR_BAD_DISCRIMINANT | (2u << 8);  // rejected_reply
  if (nw < 5) return XDRG_ERR_OVERFLOW_GET;
  h.w[XDRG_RPC_W_WHY] = pre[4];
  c.p += 20;
  return 0;
}

// One wave per workgroup, 64 consecutive messages.  Their bytes are one
// contiguous stretch of the stream: the wave loads up to kWinBytes of it
// into LDS with coalesced 16-byte loads, then every lane walks its header
// from LDS (words past the window are read from global memory).  The 64
// 64-byte records are transposed through LDS and stored as coalesced
// 16-byte chunks.
constexpr uint32_t kWinBytes = 12288;

template <bool CLIENT>
__global__ __launch_bounds__(64) void k_rpc_hdr(const uint8_t *__restrict__ s, uint64_t len,
                                                const uint64_t *__restrict__ offs, uint64_t n,
                                                const xdrg_rpc_proc *__restrict__ procs,
                                                uint32_t nprocs, const uint32_t *__restrict__ xids,
                                                xdrg_rpc_hdr *__restrict__ out) {
  __shared__ u32x4 win4[kWinBytes / 16];
  const uint32_t lane = threadIdx.x;
  const uint64_t b0 = static_cast<uint64_t>(blockIdx.x) * 64u;
  const uint64_t i = b0 + lane;
  const uint32_t nmsg = static_cast<uint32_t>(min<uint64_t>(64, n - b0));
  const uint64_t m0 = i < n ? offs[i] : 0, m1 = i < n ? offs[i + 1] : 0;
  // the wave's stretch [lo, hi) and its window (16-byte aligned stream)
  const uint64_t lo = __shfl(m0, 0, 64), hi = __shfl(m1, nmsg - 1, 64);
  uint64_t wb = lo & ~15ull, we = wb;
  if ((reinterpret_cast<uintptr_t>(s) & 15u) == 0 && lo <= hi && hi <= len) {
    we = min(min(hi, wb + kWinBytes), len);
    we = wb + ((we - wb) & ~15ull);
    const uint32_t nc = static_cast<uint32_t>((we - wb) >> 4);
    const u32x4 *src = reinterpret_cast<const u32x4 *>(s + wb);
    for (uint32_t c = lane; c < nc; c += 64) win4[c] = src[c];
  }
  __syncthreads();
  hdr_out h;
  h.end = m1;
  uint32_t err = 0;
  if (i < n) {
    if (m1 > len || m1 < m0 + 4 || (m0 & 3u)) {
      err = XDRG_ERR_MSG_MISMATCH;  // not a message of an xdrg_index_msgs index
    } else if ((m1 - m0) & 3u) {
      err = XDRG_ERR_SIZE_NOT_MULT4;  // xdr_generic_get ctor, marshal.h:157-159
    } else {
      cursor c;
      c.s = s;
      c.win = reinterpret_cast<const uint32_t *>(win4);
      c.wb = wb;
      c.we = we;
      c.p = m0 + 4;
      c.e = m1;
      const uint64_t pw = (m1 - m0 - 4) >> 2;
      const uint32_t nw = pw < 8 ? static_cast<uint32_t>(pw) : 8u;
      uint32_t pre[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) pre[k] = k < nw ? bswap(c.raw(c.p + 4u * k)) : 0u;
      err = walk(c, pre, nw, h);
      h.body_off = c.p;
    }
    if (err) {  // a malformed header keeps only action, err, the union site and end
      h = hdr_out{};
      h.end = m1;
      h.w[0] = err >> 8;
      err &= 0xffu;
    }
  }
  h.err = err;
  if (!CLIENT) {
    // rpc_server_base::dispatch (server.cc:84-107), then call_dispatch
    // (srpc.h:125-127)
    if (err) h.action = XDRG_RPC_DROP_MALFORMED;
    else if (h.mtype != CALL) h.action = XDRG_RPC_DROP_NONCALL;
    else if (h.w[XDRG_RPC_W_RPCVERS] != 2) h.action = XDRG_RPC_RPC_MISMATCH;
    else {
      const uint32_t P = h.w[XDRG_RPC_W_PROG], V = h.w[XDRG_RPC_W_VERS], Q = h.w[XDRG_RPC_W_PROC];
      const uint32_t lp = lower(procs, nprocs, P, 0, 0, 1);
      if (lp == nprocs || procs[lp].prog != P) {
        h.action = XDRG_RPC_PROG_UNAVAIL;
      } else {
        const uint32_t lv = lower(procs, nprocs, P, V, 0, 2);
        if (lv == nprocs || procs[lv].prog != P || procs[lv].vers != V) {
          h.action = XDRG_RPC_PROG_MISMATCH;
          h.w[XDRG_RPC_W_LOW] = procs[lp].vers;  // servers_[prog].cbegin()
          h.w[XDRG_RPC_W_HIGH] = procs[upper_prog(procs, nprocs, P) - 1].vers;  // crbegin()
        } else {
          const uint32_t lq = lower(procs, nprocs, P, V, Q, 3);
          const bool hit = lq < nprocs && procs[lq].prog == P && procs[lq].vers == V &&
                           procs[lq].proc == Q && !(procs[lq].flags & XDRG_RPC_PROC_IFACE_ONLY);
          h.action = hit ? XDRG_RPC_DISPATCH : XDRG_RPC_PROC_UNAVAIL;
        }
      }
    }
  } else {
    // archive(g, hdr); check_call_hdr(hdr); xid test (srpc.h:61-66)
    if (err) h.action = XDRG_RPCR_MALFORMED;
    else if (h.mtype != REPLY) h.action = XDRG_RPCR_NOT_REPLY;
    else if (h.w[XDRG_RPC_W_REPLY_STAT] == MSG_ACCEPTED)
      h.action = h.w[XDRG_RPC_W_STAT] == SUCCESS ? XDRG_RPCR_OK : XDRG_RPCR_ACCEPT_STAT;
    else
      h.action = h.w[XDRG_RPC_W_STAT] == AUTH_ERROR ? XDRG_RPCR_AUTH_STAT
                                                    : XDRG_RPCR_RPCVERS_MISMATCH;
    if (h.action == XDRG_RPCR_OK && xids && xids[i] != h.xid) h.action = XDRG_RPCR_BAD_XID;
  }
  // transpose the 64 records through LDS, then coalesced 16-byte stores
  __syncthreads();  // window fully consumed
  win4[4 * lane + 0] = u32x4{h.xid, h.action | (h.err << 16) | (h.mtype << 24), h.w[0], h.w[1]};
  win4[4 * lane + 1] = u32x4{h.w[2], h.w[3], h.w[4], h.w[5]};
  win4[4 * lane + 2] = u32x4{h.w[6], h.w[7], h.cred_len, h.verf_len};
  win4[4 * lane + 3] = u32x4{static_cast<uint32_t>(h.body_off), static_cast<uint32_t>(h.body_off >> 32),
                             static_cast<uint32_t>(h.end), static_cast<uint32_t>(h.end >> 32)};
  __syncthreads();
  u32x4 *o = reinterpret_cast<u32x4 *>(out + b0);
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q) {
    const uint32_t c = q * 64u + lane;
    if (c < 4u * nmsg) o[c] = win4[c];
  }
}

// -------------------------------------------------------------- replies
// Message bytes (mark included) of a header's error reply (server.cc:8-67).
__device__ __forceinline__ uint32_t reply_bytes(uint32_t action) {
  switch (action) {
    case XDRG_RPC_RPC_MISMATCH:
    case XDRG_RPC_PROG_UNAVAIL:
    case XDRG_RPC_PROC_UNAVAIL:
    case XDRG_RPC_GARBAGE_ARGS:
    case XDRG_RPC_SYSTEM_ERR: return 28;
    case XDRG_RPC_PROG_MISMATCH: return 36;
    case XDRG_RPC_AUTH_ERROR: return 24;
    default: return 0;
  }
}

__device__ __forceinline__ uint32_t block_sum256(uint32_t v, uint32_t *ws) {
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) ws[wid] = v;
  __syncthreads();
  return ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(256) void k_rpc_reply_sizes(const xdrg_rpc_hdr *__restrict__ hdrs,
                                                         uint64_t n,
                                                         unsigned long long *__restrict__ bsum) {
  __shared__ uint32_t ws[4];
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  const uint32_t b = i < n ? reply_bytes(hdrs[i].action) : 0u;
  const uint32_t t = block_sum256(b, ws);
  if (threadIdx.x == 0) bsum[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_rpc_reply_emit(
    const xdrg_rpc_hdr *__restrict__ hdrs, uint64_t n, uint8_t *__restrict__ out, uint64_t cap,
    uint64_t *__restrict__ offsets, const unsigned long long *__restrict__ bsum,
    unsigned long long *err) {
  __shared__ uint32_t ws[4];
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  const xdrg_rpc_hdr h = i < n ? hdrs[i] : xdrg_rpc_hdr{};
  const uint32_t b = i < n ? reply_bytes(h.action) : 0u;
  uint32_t incl = b;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= static_cast<uint32_t>(o)) incl += y;
  }
  if (lane == 63) ws[wid] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (uint32_t w = 0; w < wid; ++w) wbase += ws[w];
  if (i >= n) return;
  const uint64_t at = bsum[blockIdx.x] + wbase + incl - b;
  offsets[i] = at;
  if (!b) return;
  if (at + b > cap) {  // xdr_generic_put::check (marshal.h:104-108)
    const unsigned long long key = (static_cast<unsigned long long>(i) << 24) |
                                   (0xffffull << 8) | XDRG_ERR_OVERFLOW_PUT;
    atomicMin(err, key);
    return;
  }
  // message_t::alloc mark (marshal.cc:15-31), then the xdr_put words
  uint32_t w[9];
  uint32_t k = 0;
  w[k++] = (b - 4u) | XDRG_MARK_LAST;
  w[k++] = h.xid;
  w[k++] = REPLY;
  if (h.action == XDRG_RPC_RPC_MISMATCH) {  // rpc_rpc_mismatch_msg, server.cc:55-68
    w[k++] = MSG_DENIED; w[k++] = RPC_MISMATCH; w[k++] = 2; w[k++] = 2;
  } else if (h.action == XDRG_RPC_AUTH_ERROR) {  // rpc_auth_error_msg, server.cc:41-53
    w[k++] = MSG_DENIED; w[k++] = AUTH_ERROR; w[k++] = h.w[XDRG_RPC_W_WHY];
  } else {  // rpc_accepted_error_msg / rpc_prog_mismatch_msg, server.cc:8-39
    w[k++] = MSG_ACCEPTED; w[k++] = 0 /* AUTH_NONE */; w[k++] = 0 /* body<> */;
    const uint32_t stat = h.action == XDRG_RPC_PROG_UNAVAIL  ? PROG_UNAVAIL
                        : h.action == XDRG_RPC_PROG_MISMATCH ? PROG_MISMATCH
                        : h.action == XDRG_RPC_PROC_UNAVAIL  ? PROC_UNAVAIL
                        : h.action == XDRG_RPC_GARBAGE_ARGS  ? GARBAGE_ARGS
                                                             : SYSTEM_ERR;
    w[k++] = stat;
    if (stat == PROG_MISMATCH) { w[k++] = h.w[XDRG_RPC_W_LOW]; w[k++] = h.w[XDRG_RPC_W_HIGH]; }
  }
  uint32_t *o = reinterpret_cast<uint32_t *>(out + at);
  for (uint32_t j = 0; j < k; ++j) o[j] = bswap(w[j]);
}

// block sums, then their exclusive scan
size_t replies_ws_half(uint64_t n) { return (((n + 255) / 256 + 1) * 8 + 255) / 256 * 256; }
size_t replies_ws_bytes(uint64_t n) { return 2 * replies_ws_half(n); }

#define HIPCHK(x)                                                             \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) return xdrg::record_hip_error(int(e_), #x);         \
  } while (0)

int hdr_launch(bool client, const void *d_stream, uint64_t len, const uint64_t *d_offsets,
               uint64_t n, const xdrg_rpc_proc *d_procs, uint32_t nprocs, const uint32_t *d_xids,
               xdrg_rpc_hdr *d_hdrs, void *stream) {
  if (n == 0) return XDRG_OK;
  if (!d_stream || !d_offsets || !d_hdrs) return XDRG_EINVAL;
  if (!client && nprocs && !d_procs) return XDRG_EINVAL;
  if (!client && nprocs > XDRG_RPC_MAX_PROCS) return XDRG_EUNSUPPORTED;
  if ((reinterpret_cast<uintptr_t>(d_stream) & 3u) || (reinterpret_cast<uintptr_t>(d_offsets) & 7u) ||
      (reinterpret_cast<uintptr_t>(d_hdrs) & 15u) || (d_procs && (reinterpret_cast<uintptr_t>(d_procs) & 15u)) ||
      (d_xids && (reinterpret_cast<uintptr_t>(d_xids) & 3u)))
    return XDRG_EALIGN;
  const uint64_t blocks = (n + 63) / 64;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint8_t *s8 = static_cast<const uint8_t *>(d_stream);
  if (client)
    k_rpc_hdr<true><<<blocks, 64, 0, s>>>(s8, len, d_offsets, n, nullptr, 0, d_xids, d_hdrs);
  else
    k_rpc_hdr<false><<<blocks, 64, 0, s>>>(s8, len, d_offsets, n, d_procs, nprocs, nullptr, d_hdrs);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

}  // namespace

extern "C" {

int xdrg_rpc_dispatch(const void *d_stream, uint64_t len, const uint64_t *d_offsets, uint64_t n,
                      const xdrg_rpc_proc *d_procs, uint32_t nprocs, xdrg_rpc_hdr *d_hdrs,
                      void *stream) {
  return hdr_launch(false, d_stream, len, d_offsets, n, d_procs, nprocs, nullptr, d_hdrs, stream);
}

int xdrg_rpc_check_replies(const void *d_stream, uint64_t len, const uint64_t *d_offsets,
                           uint64_t n, const uint32_t *d_xids, xdrg_rpc_hdr *d_hdrs,
                           void *stream) {
  return hdr_launch(true, d_stream, len, d_offsets, n, nullptr, 0, d_xids, d_hdrs, stream);
}

size_t xdrg_rpc_replies_workspace_size(uint64_t n) { return replies_ws_bytes(n); }

int xdrg_rpc_replies(const xdrg_rpc_hdr *d_hdrs, uint64_t n, void *d_out, uint64_t out_capacity,
                     uint64_t *d_offsets, void *d_workspace, size_t workspace_bytes,
                     xdrg_status *d_status, void *stream) {
  if (!d_offsets || !d_status || (n && !d_hdrs)) return XDRG_EINVAL;
  if ((reinterpret_cast<uintptr_t>(d_out) & 3u) || (reinterpret_cast<uintptr_t>(d_offsets) & 7u) ||
      (reinterpret_cast<uintptr_t>(d_hdrs) & 15u))
    return XDRG_EALIGN;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n == 0) {
    HIPCHK(static_cast<hipError_t>(xdrg::fill32(d_offsets, 0u, 2, s)));
    HIPCHK(static_cast<hipError_t>(xdrg::fill32(&d_status->total_bytes, 0u, 2, s)));
    return XDRG_OK;
  }
  if (!d_workspace || workspace_bytes < replies_ws_bytes(n)) return XDRG_ESPACE;
  if (!d_out && out_capacity) return XDRG_EINVAL;
  const uint64_t nb = (n + 255) / 256;
  if (nb > 0xffffffffull) return XDRG_EUNSUPPORTED;
  auto *bsum = static_cast<unsigned long long *>(d_workspace);
  auto *bbase = bsum + replies_ws_half(n) / 8;
  k_rpc_reply_sizes<<<nb, 256, 0, s>>>(d_hdrs, n, bsum);
  HIPCHK(hipGetLastError());
  const int rc = xdrg::launch_block_scan(bsum, bbase, uint32_t(nb), d_status, d_offsets, n, stream);
  if (rc != XDRG_OK) return rc;
  k_rpc_reply_emit<<<nb, 256, 0, s>>>(d_hdrs, n, static_cast<uint8_t *>(d_out), out_capacity,
                                      d_offsets, bbase,
                                      reinterpret_cast<unsigned long long *>(&d_status->first_error));
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

}  // extern "C"
