// MI355X (gfx950) kernels and C-ABI entry points of the batched XDR engine.
//
// Kernels
//   k_fixed_reg   fixed-size, identity-layout schemas (native offsets ==
//                 wire offsets, e.g. rec128): every lane streams 16-byte
//                 chunks; each output word is one v_perm_b32 of the aligned
//                 8-byte pair it lives in (swap32 / swap64 of
//                 xdrpp/endian.h:56-68 and the high-word-first order of
//                 marshal_swap::put64/get64, xdrpp/marshal.h:65-80).  Pure
//                 HBM streaming: 16 B/lane loads and stores, no LDS.
//   k_fixed_lds   fixed-size, general layout (e.g. numerics: 56 B native,
//                 44 B wire): a workgroup stages a tile of records in LDS
//                 with coalesced 16-byte loads, then every lane assembles
//                 16 bytes of the output stream from per-word term programs
//                 and stores them coalesced.
//   k_var_size    variable plans: one record per lane walks the plan and
//                 computes xdr_size (xdrpp/types.h:240-244) + block sums.
//   k_scan_blocks exclusive scan of the block sums (one workgroup).
//   k_var_encode  block-local scan of the record sizes -> record offsets,
//                 then one record per lane interprets the plan and writes
//                 the record (xdr_generic_put, xdrpp/marshal.h:84-137).
//   k_var_decode  one record per lane, record offsets from the index
//                 (xdr_generic_get, xdrpp/marshal.h:142-211).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "plan.h"

using namespace xdrg;

namespace {

thread_local char g_hip_err[256] = "";

// This host thread's word of mapped, pinned host memory for a verdict the
// host waits for (the record index's speculative walk): the kernel writes
// it, the host reads it after the stream synchronises -- no device-to-host
// copy in the stream.  Allocated once per thread (never freed: a few bytes
// per thread that indexes); nullptr when the allocation fails.
uint32_t *host_verdict_word() {
  static thread_local uint32_t *w = nullptr;
  static thread_local bool tried = false;
  if (!tried) {
    tried = true;
    void *p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) == hipSuccess)
      w = static_cast<uint32_t *>(p);
  }
  return w;
}

int hip_fail(hipError_t e, const char *what) {
  snprintf(g_hip_err, sizeof g_hip_err, "%s: %s", what, hipGetErrorString(e));
  return XDRG_EHIP;
}
#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t e_ = (x);                            \
    if (e_ != hipSuccess) return hip_fail(e_, #x);  \
  } while (0)

}  // namespace

#include "kernels.h"
#include "var_kernels.h"
#include "index_kernels.h"
#include "elem_kernels.h"
#include "sub_kernels.h"
using namespace xdrg::dev;

namespace {

// Packed element areas (oracle/xdr_oracle.c rec_ebytes): the bytes the
// element arrays of the record at [p, b) take, each rounded up to 8 -- a
// walk of its lengths, counts and discriminants (no value checks) that
// stops where the structure stops parsing.  Jumps and arms go forward only,
// so one wave-uniform sweep of the ops reaches every op a lane can reach
// (interp_walk); every lane of the wave calls it, `on` or not.
template <class RD>
__device__ uint64_t ebytes_sweep(const xdrg_op *ops, uint32_t nops, const uint32_t *__restrict__ table,
                                 RD &rd, uint64_t p, uint64_t b, bool on) {
  constexpr uint32_t kDone = 0xffffffffu;
  uint64_t E = 0;
  uint32_t pc = on ? 0u : kDone;
  for (uint32_t upc = 0; upc < nops; ++upc) {
    if (!__any(pc == upc)) continue;
    const xdrg_op op = load_op(ops, upc);
    if (pc != upc) continue;
    const uint64_t rem = b - p;
    switch (op.kind) {
    case XDRG_OP_END: pc = kDone; break;
    case XDRG_OP_JUMP: pc = op.arg0; break;
    case XDRG_OP_U64:
      if (rem < 8) { pc = kDone; break; }
      p += 8; ++pc; break;
    case XDRG_OP_OPAQUE:
      if (rem < op.arg0) { pc = kDone; break; }
      p += (op.arg0 + 3u) & ~3u; ++pc; break;
    case XDRG_OP_U32: case XDRG_OP_BOOL: case XDRG_OP_ENUM:
      if (rem < 4) { pc = kDone; break; }
      p += 4; ++pc; break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      if (rem < 4) { pc = kDone; break; }
      const uint32_t v = bswap32(rd(p));
      p += 4;
      if (v > op.arg0 || v > b - p) { pc = kDone; break; }
      p += (static_cast<uint64_t>(v) + 3u) & ~3ull; ++pc; break;
    }
    case XDRG_OP_UNION: {
      if (rem < 4) { pc = kDone; break; }
      const int t = union_target(op, table, bswap32(rd(p)));
      p += 4;
      pc = t < 0 ? kDone : static_cast<uint32_t>(t);
      break;
    }
    case XDRG_OP_VECTOR: {
      if (rem < 4) { pc = kDone; break; }
      const uint32_t v = bswap32(rd(p));
      p += 4;
      if (v > op.arg0) { pc = kDone; break; }
      const uint64_t left = b - p, w = op.arg3;
      E += (min<uint64_t>(v, left / w + 1) * op.arg1 + 7u) & ~7ull;
      if (left < static_cast<uint64_t>(v) * w) { pc = kDone; break; }
      p += static_cast<uint64_t>(v) * w;
      pc += 1 + op.arg2;
      break;
    }
    default: ++pc; break;
    }
  }
  return E;
}

// -------------------------------------------------------- var: size pass
// xdr_traits<T>::serial_size per record and bad discriminants
// (gen_hh.cc:639-648).  The stack budget is a put-side check
// (marshal.h:129-136) and is applied by k_var_encode.
// All var kernels walk the plan with a wave-uniform schedule: jumps are
// forward-only, so the plan is a DAG in pc order and one sweep
// upc = 0..nops-1 visits every op a lane can reach.  At each upc the op is
// read through the scalar cache and dispatched with scalar branches; only
// the lanes whose own pc equals upc do the field work (and jump forward).
constexpr uint32_t kPcDone = 0xffffffffu;

// One 64-thread workgroup = 64 consecutive records.  The native records are
// staged in LDS with coalesced 16-byte loads, so the walk reads fields from
// LDS instead of issuing one dependent global load per op.
// DEPTH: also the deepest class/container level the record's walk enters
// (depth_checker, xdrpp/depth_checker.h:41-54), into depths[r].
template <bool TILE, bool DEPTH = false>
__global__ __launch_bounds__(64) void k_var_size(const uint8_t *__restrict__ native, uint64_t n,
                                                 uint32_t stride, const xdrg_op *__restrict__ ops,
                                                 uint32_t nops, const uint32_t *__restrict__ table,
                                                 uint32_t *__restrict__ sizes,
                                                 unsigned long long *__restrict__ block_sums,
                                                 uint32_t mark, unsigned long long *err,
                                                 uint32_t *__restrict__ depths = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
  const uint32_t lane = threadIdx.x;
  const uint64_t wr0 = static_cast<uint64_t>(blockIdx.x) * 64u;
  const uint64_t r = wr0 + lane;
  const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(64, n - wr0));
  if (TILE) {
    const uint32_t nbytes = nrec * stride;
    const uint8_t *nsrc = native + wr0 * stride;
    if ((reinterpret_cast<uintptr_t>(nsrc) & 15u) == 0) {
      stage_tile(tile, nsrc, nbytes, lane, 64u);
    } else {
      for (uint32_t i = lane; i < nbytes / 4u; i += 64u)
        reinterpret_cast<uint32_t *>(tile)[i] = reinterpret_cast<const uint32_t *>(nsrc)[i];
    }
  }
  wave_sync();
  const uint8_t *nat = TILE ? tile + lane * stride : native + r * stride;
  uint64_t s = mark;  // record-marked batches: the message's 4-byte mark
  uint32_t pc = r < n ? 0u : kPcDone, bad_op = kPcDone, dmax = 0;
  for (uint32_t upc = 0; upc < nops; ++upc) {
    if (!__any(pc == upc)) continue;
    const xdrg_op op = load_op(ops, upc);
    if (pc != upc) continue;
    if (DEPTH && op.kind != XDRG_OP_JUMP && op.kind != XDRG_OP_END) {
      dmax = max(dmax, static_cast<uint32_t>(op.depth));
      // a non-empty xvector / pointer enters its element's levels
      if (op.kind == XDRG_OP_VECTOR && *reinterpret_cast<const uint32_t *>(nat + op.noff + 8))
        for (uint32_t k = 1; k <= op.arg2; ++k) dmax = max(dmax, static_cast<uint32_t>(load_op(ops, upc + k).depth));
    }
    switch (op.kind) {
    case XDRG_OP_END: pc = kPcDone; break;
    case XDRG_OP_JUMP: pc = op.arg0; break;
    case XDRG_OP_U64: s += 8; ++pc; break;
    case XDRG_OP_OPAQUE: s += (op.arg0 + 3u) & ~3u; ++pc; break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
      s += 4u + ((static_cast<uint64_t>(*reinterpret_cast<const uint32_t *>(nat + op.noff + 8)) + 3u) & ~3ull);
      ++pc;
      break;
    case XDRG_OP_UNION: {
      const int t = union_target(op, table, *reinterpret_cast<const uint32_t *>(nat + op.noff));
      s += 4;
      if (t < 0) { bad_op = upc; pc = kPcDone; }
      else pc = static_cast<uint32_t>(t);
      break;
    }
    case XDRG_OP_VECTOR:  // count word + count fixed-size elements (arg3 = element wire bytes)
      s += 4ull + static_cast<uint64_t>(*reinterpret_cast<const uint32_t *>(nat + op.noff + 8)) * op.arg3;
      pc = upc + 1 + op.arg2;
      break;
    default: s += 4; ++pc; break;
    }
  }
  uint32_t size = 0;
  if (r < n) {
    if (bad_op != kPcDone) {
      report(err, r, bad_op, XDRG_ERR_BAD_DISCRIMINANT);
      size = kSizeErr;
    } else if (s >= kSizeErr) {
      report(err, r, 0, XDRG_ERR_OVERFLOW_PUT);
      size = kSizeErr;
    } else {
      size = static_cast<uint32_t>(s);
    }
    if (sizes) sizes[r] = size;
    if (DEPTH) depths[r] = dmax;
  }
  unsigned long long v = (size & kSizeErr) ? 0ull : size;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (block_sums && lane == 0) block_sums[blockIdx.x] = v;
}

// Exclusive scan of nb block sums in place; writes the total to
// status->total_bytes and offsets[n].  Workgroups of 16 waves.  A tile's
// loads are coalesced into LDS; each thread scans SUB contiguous values
// serially, the thread totals take one 64-bit wave scan, the 16 wave totals
// one more pass.  With nb <= kScanMulti every 1024-value tile has its own
// workgroup, which first sums all values before its tile (coalesced, its
// own value's load and up to 16 more per thread in flight at once) -- no
// inter-workgroup communication, one memory round trip per workgroup for
// nb <= 16K (1M records).  Larger nb: one workgroup walks 4096-value tiles
// carrying the running total.  (Measured on MI355X: per-row wave scans of
// 16 x 1024 values took ~12 us for any nb; the single-workgroup tile walk
// ~3.5 us per tile; 4096-value tiles per workgroup 7.7 us for 16K values.)
constexpr uint32_t kScanNT = 1024, kScanSub = 4, kScanTile = kScanNT * kScanSub;
constexpr uint32_t kScanMulti = 64u * kScanNT;

template <uint32_t SUB = kScanSub>
__device__ __forceinline__ unsigned long long scan_tile(const unsigned long long *in,
                                                        unsigned long long *out,
                                                        uint64_t t0, uint32_t nb,
                                                        unsigned long long carry,
                                                        unsigned long long *buf,
                                                        unsigned long long *wtot) {
  constexpr uint32_t NW = kScanNT / 64;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  auto sk = [](uint32_t e) { return e + (e >> 5); };  // skew: fewer bank conflicts
#pragma unroll
  for (uint32_t k = 0; k < SUB; ++k) {
    const uint32_t e = k * kScanNT + tid;
    buf[sk(e)] = t0 + e < nb ? in[t0 + e] : 0ull;
  }
  __syncthreads();
  unsigned long long x[SUB], tsum = 0;
#pragma unroll
  for (uint32_t k = 0; k < SUB; ++k) {
    x[k] = buf[sk(SUB * tid + k)];
    tsum += x[k];
  }
  unsigned long long incl = tsum;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(incl, o, 64);
    if (lane >= static_cast<uint32_t>(o)) incl += y;
  }
  if (lane == 63) wtot[wid] = incl;
  __syncthreads();
  unsigned long long wbase = 0, all = 0;
#pragma unroll
  for (uint32_t w = 0; w < NW; ++w) {
    const unsigned long long t = wtot[w];
    if (w < wid) wbase += t;
    all += t;
  }
  unsigned long long run = carry + wbase + incl - tsum;
#pragma unroll
  for (uint32_t k = 0; k < SUB; ++k) {
    buf[sk(SUB * tid + k)] = run;
    run += x[k];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < SUB; ++k) {
    const uint32_t e = k * kScanNT + tid;
    if (t0 + e < nb) out[t0 + e] = buf[sk(e)];
  }
  __syncthreads();  // buf / wtot reused by the next tile
  return carry + all;
}

// MULTI reads `in` and writes `out` (distinct: other workgroups still read
// `in`); the single-workgroup walk may scan in place.
template <bool MULTI>
__global__ __launch_bounds__(1024) void k_scan_blocks(const unsigned long long *in,
                                                      unsigned long long *out, uint32_t nb,
                                                      xdrg_status *status,
                                                      uint64_t *__restrict__ offsets, uint64_t n) {
  __shared__ unsigned long long buf[kScanTile + kScanTile / 32];
  __shared__ unsigned long long wtot[kScanNT / 64];
  const uint32_t tid = threadIdx.x;
  unsigned long long carry = 0;
  if (MULTI) {
    // this workgroup's 1024-value tile; its carry = the sum of every value
    // before it, up to 16 loads per thread in flight
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kScanNT;
    unsigned long long part = 0;
    for (uint64_t j0 = 0; j0 < t0; j0 += 16u * kScanNT) {
      unsigned long long q[16];
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) {
        const uint64_t j = j0 + k * kScanNT + tid;
        q[k] = j < t0 ? in[j] : 0ull;
      }
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) part += q[k];
    }
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if ((tid & 63) == 0) wtot[tid >> 6] = part;
    __syncthreads();
#pragma unroll
    for (uint32_t w = 0; w < kScanNT / 64; ++w) carry += wtot[w];
    __syncthreads();
    carry = scan_tile<1>(in, out, t0, nb, carry, buf, wtot);
    if (tid == 0 && blockIdx.x == gridDim.x - 1) {
      status->total_bytes = carry;
      if (offsets) offsets[n] = carry;
    }
    return;
  }
  for (uint64_t t0 = 0; t0 < nb; t0 += kScanTile) carry = scan_tile(in, out, t0, nb, carry, buf, wtot);
  if (tid == 0) {
    status->total_bytes = carry;
    if (offsets) offsets[n] = carry;
  }
}

// ------------------------------------------------------------ var: encode
__global__ __launch_bounds__(256) void k_var_encode(
    const uint8_t *__restrict__ native, uint64_t n, uint32_t stride, const uint8_t *__restrict__ heap,
    uint64_t heap_len, uint8_t *__restrict__ xdr, uint64_t cap, uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ sizes, const unsigned long long *__restrict__ block_base,
    const xdrg_op *__restrict__ ops, uint32_t nops, const uint32_t *__restrict__ table,
    uint32_t stack_limit, uint32_t mark, unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  __shared__ unsigned long long wsum[4];
  load_ops(sops, ops, nops);
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t sz = r < n ? sizes[r] : 0u;
  // block-local exclusive scan (wave scan + wave totals)
  unsigned long long v = (sz & kSizeErr) ? 0ull : sz;
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long x = __shfl_up(incl, o, 64);
    if (lane >= static_cast<uint32_t>(o)) incl += x;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  const uint64_t off = block_base[blockIdx.x * 4u + wid] + incl - v;  // 64-record block bases
  if (r >= n) return;
  offsets[r] = off;
  if (sz & kSizeErr) return;  // size pass reported this record

  const uint8_t *nat = native + r * stride;
  uint64_t pos = off;
  if (mark) {  // the message's record mark (message_t::alloc, marshal.cc:15-31)
    if (4 > cap - min(pos, cap)) { report(err, r, kOpRecordLevel, XDRG_ERR_OVERFLOW_PUT); return; }
    st32(xdr + pos, mark_word(sz - 4u));
    pos += 4;
  }
  uint32_t pc = 0;
  for (;;) {
    const xdrg_op &op = sops[pc];
    if (op.kind == XDRG_OP_END) break;
    if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; continue; }
    if (op.depth > stack_limit) {  // marshal.h:131-132
      report(err, r, pc, XDRG_ERR_STACK_PUT);
      return;
    }
    uint64_t need;
    uint32_t len = 0;
    switch (op.kind) {
    case XDRG_OP_U64: need = 8; break;
    case XDRG_OP_OPAQUE: need = op.arg0; break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
      len = ld32(nat + op.noff + 8);
      need = 4ull + len;
      break;
    default: need = 4; break;
    }
    if (need > cap - min(pos, cap)) {  // check(n), marshal.h:104-108
      report(err, r, pc, XDRG_ERR_OVERFLOW_PUT);
      return;
    }
    uint32_t *o = reinterpret_cast<uint32_t *>(xdr + pos);
    switch (op.kind) {
    case XDRG_OP_U32: case XDRG_OP_ENUM:
      o[0] = bswap32(ld32(nat + op.noff)); pos += 4; ++pc; break;
    case XDRG_OP_BOOL:
      o[0] = nat[op.noff] ? 0x01000000u : 0u; pos += 4; ++pc; break;
    case XDRG_OP_U64:
      o[0] = bswap32(ld32(nat + op.noff + 4));
      o[1] = bswap32(ld32(nat + op.noff));
      pos += 8; ++pc; break;
    case XDRG_OP_OPAQUE: {
      const uint32_t L = op.arg0, nw = (L + 3u) >> 2;
      for (uint32_t k = 0; k < nw; ++k) {
        uint32_t w = unaligned_word(nat, stride, op.noff + 4ull * k);
        if (4 * k + 4 > L) w &= keep_mask(L - 4 * k);
        o[k] = w;
      }
      pos += 4ull * nw; ++pc; break;
    }
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      const uint64_t hoff = *reinterpret_cast<const uint64_t *>(nat + op.noff);
      const uint32_t nw = (len + 3u) >> 2;
      o[0] = bswap32(len);
      for (uint32_t k = 0; k < nw; ++k) {
        uint32_t w = unaligned_word(heap, heap_len, hoff + 4ull * k);
        if (4 * k + 4 > len) w &= keep_mask(len - 4 * k);
        o[1 + k] = w;
      }
      pos += 4ull + 4ull * nw; ++pc; break;
    }
    case XDRG_OP_UNION: {
      const uint32_t d = ld32(nat + op.noff);
      o[0] = bswap32(d);
      pos += 4;
      pc = static_cast<uint32_t>(union_target(op, table, d));  // validated by k_var_size
      break;
    }
    case XDRG_OP_VECTOR: {
      const uint64_t eoff = *reinterpret_cast<const uint64_t *>(nat + op.noff);
      const uint32_t cnt = ld32(nat + op.noff + 8);
      o[0] = bswap32(cnt);
      pos += 4;
      uint32_t at = static_cast<uint32_t>(pos - off);
      auto put = [&](uint32_t a, uint32_t w) { st32(xdr + off + a, w); };
      if (!enc_vector_elems(sops, pc + 1, op.arg2, heap, heap_len, eoff, cnt, op.arg1, pos, cap, at,
                            stack_limit, r, err, put))
        return;
      pc += 1 + op.arg2;
      break;
    }
    default: ++pc; break;
    }
  }
}

// ------------------------------------------------------------ var: decode
// Record r = xdr_from_opaque(stream[off[r], off[r+1]), r): fields walk in
// plan order with check() before every read; the native record is
// zero-filled first.  The decoded heap is the stream itself (the host
// copies it to heap_out): a payload's xdrg_bytes_ref holds its stream offset.
__global__ __launch_bounds__(256) void k_var_decode(
    const uint8_t *__restrict__ xdr, uint64_t len, const uint64_t *__restrict__ offsets, uint64_t n,
    uint8_t *__restrict__ native, uint32_t stride, const xdrg_op *__restrict__ ops, uint32_t nops,
    const uint32_t *__restrict__ table, uint32_t stack_limit, uint8_t *__restrict__ heap,
    uint64_t ebase, uint32_t F, uint32_t mark, uint32_t packed, unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  load_ops(sops, ops, nops);
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t a = r < n ? offsets[r] : 0u, b = r < n ? offsets[r + 1] : 0u;
  uint64_t ecur = ebase + static_cast<uint64_t>(F) * a;  // this record's element arrays
  uint64_t eend = ebase + static_cast<uint64_t>(F) * b;
  if (packed) {  // ... packed with its wave's (var_kernels.h packed_area)
    const bool bad = r < n && (b < a || b > len);
    const bool on = r < n && !bad && a + mark <= b;
    auto rd = [&](uint64_t q) { return ld32(xdr + q); };
    const uint64_t e = ebytes_sweep(sops, nops, table, rd, a + mark, b, on);
    packed_area(on ? min(e, ebudget(F, a, b)) : 0u, bad, rl64(a, 0), ebase, F, ecur, eend);
  }
  if (r >= n) return;
  if (r == n - 1 && b != len) report(err, n, kOpRecordLevel, XDRG_ERR_TRAILING);
  if (b < a || b > len) { report(err, r, 0, XDRG_ERR_OVERFLOW_GET); return; }
  if (mark) {  // xdr_from_msg: the message read_message framed (srpc.cc:29-55)
    const uint32_t c = b - a < 4 ? XDRG_ERR_MSG_EOF : mark_code(ld32(xdr + a), b - a - 4);
    if (c) { report(err, r, kOpRecordLevel, c); return; }
  }
  if ((b - a) & 3u) { report(err, r, kOpRecordLevel, XDRG_ERR_SIZE_NOT_MULT4); return; }
  uint8_t *nat = native + r * stride;
  for (uint32_t k = 0; k < stride / 4; ++k) st32(nat + 4 * k, 0u);
  uint64_t p = a + mark;
  uint32_t pc = 0;
  for (;;) {
    const xdrg_op &op = sops[pc];
    if (op.kind == XDRG_OP_END) break;
    if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; continue; }
    if (op.depth > stack_limit) { report(err, r, pc, XDRG_ERR_STACK_GET); return; }
    const uint64_t rem = b - p;
    switch (op.kind) {
    case XDRG_OP_U32:
      if (rem < 4) goto overflow;
      st32(nat + op.noff, bswap32(ld32(xdr + p))); p += 4; ++pc; break;
    case XDRG_OP_ENUM: {
      if (rem < 4) goto overflow;
      const uint32_t v = bswap32(ld32(xdr + p));
      st32(nat + op.noff, v); p += 4;
      if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, v)) {
        report(err, r, pc, XDRG_ERR_INVALID_ENUM); return;
      }
      ++pc; break;
    }
    case XDRG_OP_BOOL:
      if (rem < 4) goto overflow;
      nat[op.noff] = ld32(xdr + p) != 0u; p += 4; ++pc; break;
    case XDRG_OP_U64:
      if (rem < 8) goto overflow;
      st32(nat + op.noff + 4, bswap32(ld32(xdr + p)));
      st32(nat + op.noff, bswap32(ld32(xdr + p + 4)));
      p += 8; ++pc; break;
    case XDRG_OP_OPAQUE: {
      const uint32_t L = op.arg0;
      if (rem < L) goto overflow;
      for (uint32_t k = 0; k < L; ++k) nat[op.noff + k] = xdr[p + k];
      if (L & 3u) {
        const uint32_t w = ld32(xdr + p + (L & ~3u));
        if (w & ~keep_mask(L & 3u)) { report(err, r, pc, XDRG_ERR_NONZERO_PAD); return; }
      }
      p += (L + 3u) & ~3u; ++pc; break;
    }
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      if (rem < 4) goto overflow;
      const uint32_t L = bswap32(ld32(xdr + p));
      p += 4;
      if (L > b - p) goto overflow;
      if (L > op.arg0) {
        report(err, r, pc,
               op.kind == XDRG_OP_STRING ? XDRG_ERR_XSTRING_BOUND : XDRG_ERR_XVECTOR_BOUND);
        return;
      }
      const uint32_t nw = (L + 3u) >> 2;
      if (L & 3u) {
        const uint32_t w = ld32(xdr + p + 4ull * (nw - 1));
        if (w & ~keep_mask(L & 3u)) { report(err, r, pc, XDRG_ERR_NONZERO_PAD); return; }
      }
      *reinterpret_cast<uint64_t *>(nat + op.noff) = p;  // the payload stays in the stream
      st32(nat + op.noff + 8, L);
      p += 4ull * nw; ++pc; break;
    }
    case XDRG_OP_UNION: {
      if (rem < 4) goto overflow;
      const uint32_t d = bswap32(ld32(xdr + p));
      p += 4;
      if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, d)) {
        report(err, r, pc, XDRG_ERR_INVALID_ENUM); return;
      }
      const int t = union_target(op, table, d);
      if (t < 0) { report(err, r, pc, XDRG_ERR_BAD_DISCRIMINANT); return; }
      st32(nat + op.noff, d);
      pc = static_cast<uint32_t>(t);
      break;
    }
    case XDRG_OP_VECTOR: {
      if (rem < 4) goto overflow;
      const uint32_t cnt = bswap32(ld32(xdr + p));
      p += 4;
      if (cnt > op.arg0) {  // check_size (types.h:486-489, 605-608)
        report(err, r, pc, (op.flags & XDRG_F_POINTER) ? XDRG_ERR_POINTER_BOUND : XDRG_ERR_XVECTOR_BOUND);
        return;
      }
      if (!elem_area_ok(ecur, eend, cnt, op.arg1, op.arg3, b - p)) goto overflow;
      *reinterpret_cast<uint64_t *>(nat + op.noff) = ecur;
      st32(nat + op.noff + 8, cnt);
      auto rd = [&](uint64_t q) { return ld32(xdr + q); };
      if (!dec_vector_elems(sops, table, pc + 1, op.arg2, cnt, op.arg1, heap + ecur, p, b,
                            stack_limit, r, err, rd, reinterpret_cast<uint32_t *>(nat + op.noff + 12)))
        return;
      ecur += static_cast<uint64_t>(cnt) * op.arg1;
      pc += 1 + op.arg2;
      break;
    }
    default: ++pc; break;
    }
  }
  if (p != b) report(err, r, kOpRecordLevel, XDRG_ERR_TRAILING);
  return;
overflow:
  report(err, r, pc, XDRG_ERR_OVERFLOW_GET);
}

// ------------------------------------------ var: the plan interpreter walk
// The walker of var_kernels.h for any plan: a wave-uniform sweep over the
// op DAG (jumps are forward-only, so one sweep upc = 0..nops-1 visits every
// op a lane can reach).  At each upc the op is read through the scalar cache
// and dispatched with scalar branches; only the lanes whose own pc equals
// upc do the field work.  Plans compiled to straight-line code (spec.cpp)
// replace this walk; the interpreter serves every plan, and any plan on a
// device where its specialized kernels are not loaded.
struct interp_walk {
  static constexpr bool kFastWalk = false;  // enc() takes the checked context only
  static constexpr bool kDirect = false;    // (launched only when 64 records fit 2^31 bytes)
  static constexpr uint32_t kMaxDepth = 0;
  static constexpr uint32_t kWords = 0;  // walks every window (no word list)
  const xdrg_op *__restrict__ ops;
  uint32_t nops;
  const uint32_t *__restrict__ table;
  bool pk = false;  // decode: packed element areas (var_kernels.h packed_area)

  __device__ bool packed() const { return pk; }
  template <class RD>
  __device__ uint64_t ebytes(RD &rd, uint64_t p, uint64_t b, bool on) const {
    return ebytes_sweep(ops, nops, table, rd, p, b, on);
  }

  template <int KMAX>
  __device__ bool enc(enc_ctx<KMAX> &c, const uint8_t *nat, bool ok) const {
    uint32_t pc = ok ? 0u : kPcDone, nslot = 0;
    for (uint32_t upc = 0; upc < nops; ++upc) {
      if (!__any(pc == upc)) continue;
      const xdrg_op op = load_op(ops, upc);
      if (pc != upc) continue;
      if (op.kind == XDRG_OP_END) { pc = kPcDone; continue; }
      if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; continue; }
      const uint32_t *nw = reinterpret_cast<const uint32_t *>(nat + op.noff);
      uint32_t blen = 0;
      uint64_t need = 4;
      if (op.kind == XDRG_OP_U64) need = 8;
      else if (op.kind == XDRG_OP_OPAQUE) need = op.arg0;
      else if (op.kind == XDRG_OP_VAROPAQUE || op.kind == XDRG_OP_STRING) {
        blen = nw[2];
        need = 4ull + blen;
      }
      if (!c.field(upc, op.depth, need)) { ok = false; pc = kPcDone; continue; }
      switch (op.kind) {
      case XDRG_OP_U32: case XDRG_OP_ENUM: c.put(bswap32(nw[0])); ++pc; break;
      case XDRG_OP_BOOL: c.put(nat[op.noff] ? 0x01000000u : 0u); ++pc; break;
      case XDRG_OP_U64:
        c.put(bswap32(nw[1]));
        c.put(bswap32(nw[0]));
        ++pc;
        break;
      case XDRG_OP_OPAQUE: {
        const uint32_t BL = op.arg0, nwd = (BL + 3u) >> 2;
        for (uint32_t k = 0; k < nwd; ++k) {
          uint32_t w = 0;
          for (uint32_t bb = 0; bb < 4u && 4u * k + bb < BL; ++bb)
            w |= static_cast<uint32_t>(nat[op.noff + 4u * k + bb]) << (8u * bb);
          c.put(w);
        }
        ++pc;
        break;
      }
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
        c.put(bswap32(blen));
        const uint64_t hsrc = *reinterpret_cast<const uint64_t *>(nw);
        if (!blen) {
        } else if (nslot < static_cast<uint32_t>(KMAX) && blen <= (1u << 30)) {
          c.slot_dyn(nslot++, hsrc, blen);
        } else {
          c.copy(hsrc, blen);
        }
        ++pc;
        break;
      }
      case XDRG_OP_UNION: {
        const uint32_t d = nw[0];
        c.put(bswap32(d));
        pc = static_cast<uint32_t>(union_target(op, table, d));  // validated by the size pass
        break;
      }
      case XDRG_OP_VECTOR: {
        const uint64_t eoff = *reinterpret_cast<const uint64_t *>(nw);
        const uint32_t cnt = nw[2];
        c.put(bswap32(cnt));
        auto put = [&](uint32_t a, uint32_t w) { c.wput(a, w); };
        if (!enc_vector_elems(ops, upc + 1, op.arg2, c.heap, c.heap_len, eoff, cnt, op.arg1, c.pos,
                              c.cap, c.at, c.stack_limit, c.r, c.err, put)) {
          ok = false;
          pc = kPcDone;
          break;
        }
        pc = upc + 1 + op.arg2;
        break;
      }
      default: ++pc; break;
      }
    }
    return ok;
  }

  template <bool RA>
  __device__ bool dec(dec_ctx<RA> &c, uint8_t *nat, bool ok) const {
    uint32_t pc = ok ? 0u : kPcDone;
    for (uint32_t upc = 0; upc < nops; ++upc) {
      if (!__any(pc == upc)) continue;
      const xdrg_op op = load_op(ops, upc);
      if (pc != upc) continue;
      if (op.kind == XDRG_OP_END) { pc = kPcDone; continue; }
      if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; continue; }
      uint32_t *nw = reinterpret_cast<uint32_t *>(nat + op.noff);
      const uint32_t need = op.kind == XDRG_OP_U64 ? 8u : op.kind == XDRG_OP_OPAQUE ? op.arg0 : 4u;
      if (!c.field(upc, op.depth, need)) { ok = false; pc = kPcDone; continue; }
      uint64_t &p = c.p;
      switch (op.kind) {
      case XDRG_OP_U32: nw[0] = bswap32(c.word()); ++pc; break;
      case XDRG_OP_ENUM: {
        const uint32_t v = bswap32(c.word());
        nw[0] = v;
        ++pc;
        if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, v)) {
          ok = c.fail(upc, XDRG_ERR_INVALID_ENUM); pc = kPcDone;
        }
        break;
      }
      case XDRG_OP_BOOL: nat[op.noff] = c.word() != 0u; ++pc; break;
      case XDRG_OP_U64:
        nw[1] = bswap32(c.rd(p));
        nw[0] = bswap32(c.rd(p + 4));
        p += 8;
        ++pc;
        break;
      case XDRG_OP_OPAQUE: {
        const uint32_t BL = op.arg0;
        for (uint32_t k = 0; k < BL; k += 4) {
          const uint32_t w = c.rd(p + k);
          for (uint32_t bb = 0; bb < 4u && k + bb < BL; ++bb) nat[op.noff + k + bb] = uint8_t(w >> (8 * bb));
        }
        ++pc;
        if ((BL & 3u) && (c.rd(p + (BL & ~3u)) & ~keep_mask(BL & 3u))) {
          ok = c.fail(upc, XDRG_ERR_NONZERO_PAD); pc = kPcDone;
        }
        p += (BL + 3u) & ~3u;
        break;
      }
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
        const uint32_t BL = bswap32(c.word());
        if (BL > c.b - p) { ok = c.fail(upc, XDRG_ERR_OVERFLOW_GET); pc = kPcDone; break; }
        if (BL > op.arg0) {
          ok = c.fail(upc, op.kind == XDRG_OP_STRING ? XDRG_ERR_XSTRING_BOUND : XDRG_ERR_XVECTOR_BOUND);
          pc = kPcDone;
          break;
        }
        if ((BL & 3u) && (c.rd(p + (BL & ~3u)) & ~keep_mask(BL & 3u))) {  // get_bytes pad check
          ok = c.fail(upc, XDRG_ERR_NONZERO_PAD); pc = kPcDone; break;
        }
        *reinterpret_cast<uint64_t *>(nat + op.noff) = p;  // the payload stays in the stream
        nw[2] = BL;
        p += (static_cast<uint64_t>(BL) + 3u) & ~3ull;
        ++pc;
        break;
      }
      case XDRG_OP_UNION: {
        const uint32_t d = bswap32(c.word());
        if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, d)) {
          ok = c.fail(upc, XDRG_ERR_INVALID_ENUM); pc = kPcDone; break;
        }
        const int t = union_target(op, table, d);
        if (t < 0) { ok = c.fail(upc, XDRG_ERR_BAD_DISCRIMINANT); pc = kPcDone; break; }
        nw[0] = d;
        pc = static_cast<uint32_t>(t);
        break;
      }
      case XDRG_OP_VECTOR: {
        const uint32_t cnt = bswap32(c.word());
        if (cnt > op.arg0) {  // check_size (types.h:486-489, 605-608)
          ok = c.fail(upc, (op.flags & XDRG_F_POINTER) ? XDRG_ERR_POINTER_BOUND : XDRG_ERR_XVECTOR_BOUND);
          pc = kPcDone;
          break;
        }
        if (!c.area(upc, cnt, op.arg1, op.arg3)) { ok = false; pc = kPcDone; break; }
        *reinterpret_cast<uint64_t *>(nat + op.noff) = c.ecur;
        nw[2] = cnt;
        if (!dec_vector_elems(ops, table, upc + 1, op.arg2, cnt, op.arg1, c.heap + c.ecur, p, c.b,
                              c.stack_limit, c.r, c.err, c.rd, &nw[3])) {
          ok = false; pc = kPcDone; break;
        }
        c.ecur += static_cast<uint64_t>(cnt) * op.arg1;
        pc = upc + 1 + op.arg2;
        break;
      }
      default: ++pc; break;
      }
    }
    return ok;
  }
};

template <int KMAX, int U>
__global__ __launch_bounds__(64) void k_var_encode_i(
    const uint8_t *__restrict__ native, uint64_t n, uint32_t stride, const uint8_t *__restrict__ heap,
    uint64_t heap_len, uint8_t *__restrict__ xdr, uint64_t cap, uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ sizes, const unsigned long long *__restrict__ block_base,
    const xdrg_op *__restrict__ ops, uint32_t nops, const uint32_t *__restrict__ table,
    uint32_t stack_limit, uint32_t C, uint32_t mark, unsigned long long *err) {
  var_encode_body<interp_walk, KMAX, U>(interp_walk{ops, nops, table}, native, n, stride, heap,
                                        heap_len, xdr, cap, offsets, sizes, block_base, stack_limit,
                                        C, mark, err);
}

template <bool COPY, bool RA = true>
__global__ __launch_bounds__(64) void k_var_decode_w(
    const uint8_t *__restrict__ xdr, uint64_t len, const uint64_t *__restrict__ offsets, uint64_t n,
    uint8_t *__restrict__ native, uint32_t stride, uint8_t *__restrict__ heap,
    const xdrg_op *__restrict__ ops, uint32_t nops, const uint32_t *__restrict__ table,
    uint32_t stack_limit, uint32_t C, uint64_t ebase, uint32_t F, uint32_t mark, uint32_t packed,
    uint32_t S, unsigned long long *err) {
  var_decode_body<interp_walk, COPY, RA>(interp_walk{ops, nops, table, packed != 0}, xdr, len, offsets, n, native,
                                         stride, heap, stack_limit, C, ebase, F, mark, S, err);
}

// ------------------------------------------- element subroutines (frame walk)
// The interpreted frame walks of sub_kernels.h (plans with element
// subroutines the generated walkers do not inline: recursive types).
template <bool DEPTH>
__global__ __launch_bounds__(256) void k_sub_size(XDRG_SUB_SIZE_PARAMS) {
  sub_size_kernel<DEPTH, rt_ops>(XDRG_SUB_SIZE_ARGS);
}
__global__ __launch_bounds__(256) void k_sub_encode(XDRG_SUB_ENCODE_PARAMS) {
  sub_encode_kernel<rt_ops>(XDRG_SUB_ENCODE_ARGS);
}
__global__ __launch_bounds__(256) void k_sub_chain(XDRG_SUB_ENCODE_PARAMS) {
  sub_chain_kernel<rt_ops>(XDRG_SUB_ENCODE_ARGS);
}
__global__ __launch_bounds__(256) void k_sub_chain_size(XDRG_SUB_SIZE_PARAMS) {
  sub_chain_size_kernel<rt_ops>(XDRG_SUB_SIZE_ARGS);
}
__global__ __launch_bounds__(256) void k_sub_decode(XDRG_SUB_DECODE_PARAMS) {
  sub_decode_kernel<rt_ops>(XDRG_SUB_DECODE_ARGS);
}

// ------------------------------------------- record marks: the index pass
// The marks of a message stream form a chain (each names the next one's
// position), so finding the messages is list ranking.  The stream is cut
// into segments of kIxSW words; a message is at most max_msg_len bytes,
// so the chain enters every segment within its first K = max_msg_len/4 + 1
// words.  Only words that read as a well-formed mark ("valid" nodes: a
// last-fragment mark of a bounded, 4-aligned size that fits the stream)
// can continue a chain; every other word ends any chain that reaches it.
//   k_ix_seg   per segment: the valid nodes (written out as a list), then
//              pointer jumping over them in LDS: the exit (entry word of
//              the next segment) and the marks passed, or "ends here", for
//              each of the K entries;
//   k_ix_up    composes F consecutive tables into one (levels until one
//              node remains);
//   k_ix_down  from the top: each node's entry and the count of messages
//              before it, which reach every segment;
//   k_ix_emit  per segment on the chain: the nodes reachable from its
//              entry (doubling over the valid-node list), ranked by
//              position, give the offsets; the word where the chain ends
//              is classified exactly as read_message would (ix_mark).
static_assert(XDRG_INDEX_MAX_MSG == 4 * (kIxSW - 1), "index window = one segment");

enum ix_state : uint32_t { IX_RUN = 0, IX_END, IX_EOF, IX_SIZE4, IX_FRAG, IX_LONG, IX_MULT4 };

__device__ __forceinline__ uint32_t ix_error(uint32_t st) {
  switch (st) {
  case IX_EOF: return XDRG_ERR_MSG_EOF;
  case IX_SIZE4: return XDRG_ERR_MSG_SIZE4;
  case IX_FRAG: return XDRG_ERR_MSG_FRAGMENT;
  case IX_LONG: return XDRG_ERR_MSG_TOO_LONG;
  default: return XDRG_ERR_SIZE_NOT_MULT4;  // xdr_from_msg of it would throw this
  }
}

// The mark at stream word w (raw = its little-endian word when it lies
// inside the stream), checked as read_message reads it (srpc.cc:29-55):
// premature EOF on the mark, the pre-swap size test, the last-fragment
// bit; then msg_sock's maxmsglen_ (msgsock.cc:99-111) and a body that ends
// past the stream.  A size that is not a multiple of 4 ends the index at
// that message: xdr_from_msg rejects it (marshal.h:152-162) and the next
// mark would not be word aligned.  *nxt = word of the next mark.
__device__ __forceinline__ uint32_t ix_mark(uint32_t raw, uint64_t w, uint64_t len, uint32_t maxlen,
                                            uint64_t *nxt) {
  const uint64_t at = 4 * w;
  if (at == len) return IX_END;
  if (at + 4 > len) return IX_EOF;
  if (raw & 3u) return IX_SIZE4;
  const uint32_t v = bswap32(raw);
  if (!(v & XDRG_MARK_LAST)) return IX_FRAG;
  const uint32_t size = v & ~XDRG_MARK_LAST;
  if (size > maxlen) return IX_LONG;
  if (len - at - 4 < size) return IX_EOF;
  if (size & 3u) return IX_MULT4;
  *nxt = w + 1 + size / 4;
  return IX_RUN;
}

// ------------------------------------- concatenated records: the index pass
// xdrg_index_records runs the same list ranking over record starts: node w
// is "a record starts at word w", its successor the word after that
// record.  rx_len parses one record from byte a -- lengths, counts and
// discriminants only, the structure xdr_generic_get would walk
// (marshal.h:142-211) -- with every check that makes its decode fail
// (bounds of strings, opaques and containers, unknown discriminants,
// unlisted values of validated enums), so a node that does not parse is a
// record the decode rejects.  RX_LONG: the record runs past a + maxlen (but
// not past the stream), beyond what one segment window can index.

// Stream words through global memory (rx_global, index_kernels.h) in the
// list ranking.  (Staging a segment's reachable window in LDS first
// measured slower on MI355X: 0.69 -> 0.96 ms for 1M recvar records, the
// occupancy it costs outweighing L2-hit latency.)  The fast path
// (rxs_walk_body) stages its segment: its walks are serial chains.

// The frames of rx_len's element subroutines (with TAIL a tail container
// replaces the top frame, sub_kernels.h sub_tail: these count the frames
// open).
// rx_reg_frames: the index's own XDRG_INDEX_FRAMES in registers, st[0] the
// top frame, pushed and popped by shifting (constant indices: no private
// memory, sub_kernels.h reg_stack); a record nested deeper is RX_LONG, left
// to the long-record walk (k_rx_long) like one past the window.
// rx_slab_frames: that walk's frames, XDRG_MAX_FRAMES of them in the index
// workspace; deeper is RX_BAD (the decode reports the stack overflow).
struct rx_frame { uint32_t left, entry, ret; };
struct rx_reg_frames {
  static constexpr uint32_t kFull = RX_LONG;
  rx_frame st[XDRG_INDEX_FRAMES];
  uint32_t fp = 0;
  __device__ __forceinline__ bool full() const { return fp == XDRG_INDEX_FRAMES; }
  __device__ __forceinline__ rx_frame &top() { return st[0]; }
  __device__ __forceinline__ void push(const rx_frame &f) {
#pragma unroll
    for (int j = XDRG_INDEX_FRAMES - 1; j > 0; --j) st[j] = st[j - 1];
    st[0] = f;
    ++fp;
  }
  __device__ __forceinline__ void pop() {
    --fp;
#pragma unroll
    for (int j = 0; j + 1 < XDRG_INDEX_FRAMES; ++j) st[j] = st[j + 1];
  }
};
struct rx_slab_frames {
  static constexpr uint32_t kFull = RX_BAD;
  rx_frame *st;
  uint32_t cap, fp = 0;
  __device__ __forceinline__ bool full() const { return fp == cap; }
  __device__ __forceinline__ rx_frame &top() { return st[fp - 1]; }
  __device__ __forceinline__ void push(const rx_frame &f) { st[fp++] = f; }
  __device__ __forceinline__ void pop() { --fp; }
};

// U: the position type (uint32_t for offsets into a staged stretch).
// TAIL: a tail container takes the frame of the element it ends (the
// long-record walk); the windows' parses count every frame, so a candidate
// start inside a long list bails at XDRG_INDEX_FRAMES instead of parsing on
// to the window's end (with it, rp_list's index took 836 ms, profiles/r05n).
template <class RD, class U = uint64_t, class FS = rx_reg_frames, bool TAIL = false>
__device__ uint32_t rx_len(const xdrg_op *__restrict__ ops, const uint32_t *__restrict__ table,
                           const RD &rd, U len, U a, uint32_t maxlen, FS st = FS{}) {
  const bool capped = static_cast<uint64_t>(a) + maxlen < len;
  const U lim = capped ? static_cast<U>(a + maxlen) : len;
  const uint32_t past = capped ? RX_LONG : RX_BAD;
  uint32_t pc = 0;
  U p = a;
  for (;;) {
    const xdrg_op &op = ops[pc];
    switch (op.kind) {
    case XDRG_OP_END:
      if (!st.fp) return static_cast<uint32_t>(p - a);
      if (st.top().left) {
        --st.top().left;
        pc = st.top().entry;
      } else {
        pc = st.top().ret;
        st.pop();
      }
      continue;
    case XDRG_OP_JUMP: pc = op.arg0; continue;
    case XDRG_OP_U64:
      if (lim - p < 8) return past;
      p += 8; ++pc; continue;
    case XDRG_OP_OPAQUE:
      if (lim - p < op.arg0) return past;
      p += (op.arg0 + 3u) & ~3u; ++pc; continue;
    case XDRG_OP_U32: case XDRG_OP_BOOL:  // any value decodes: no load
      if (lim - p < 4) return past;
      p += 4; ++pc; continue;
    case XDRG_OP_ENUM:
      if (op.flags & XDRG_F_VALIDATE) break;
      if (lim - p < 4) return past;
      p += 4; ++pc; continue;
    default: break;
    }
    if (lim - p < 4) return past;
    const uint32_t v = bswap32(rd(p));
    p += 4;
    switch (op.kind) {
    case XDRG_OP_ENUM:
      if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, v)) return RX_BAD;
      ++pc;
      break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
      if (v > op.arg0) return RX_BAD;
      if (lim - p < v) return past;
      p += static_cast<U>((static_cast<uint64_t>(v) + 3u) & ~3ull);
      ++pc;
      break;
    case XDRG_OP_UNION: {
      if ((op.flags & XDRG_F_VALIDATE) && !enum_ok(table, op.arg0, op.arg1, v)) return RX_BAD;
      const int t = union_target(op, table, v);
      if (t < 0) return RX_BAD;
      pc = static_cast<uint32_t>(t);
      break;
    }
    case XDRG_OP_VECTOR:
      if (v > op.arg0) return RX_BAD;
      if (!(op.flags & XDRG_F_SUB)) {
        const uint64_t b = static_cast<uint64_t>(v) * op.arg3;
        if (static_cast<uint64_t>(lim - p) < b) return past;
        p += static_cast<U>(b);
        pc += 1 + op.arg2;
      } else if (!v) {
        ++pc;
      } else if (TAIL && st.fp && st.top().left == 0 && sub_tail(ops, pc)) {
        // a tail container takes the frame of the element it ends, and its
        // return pc (sub_kernels.h sub_tail): a linked list parses in one frame
        st.top() = rx_frame{v - 1, op.arg4, st.top().ret};
        pc = op.arg4;
      } else {
        if (st.full()) return FS::kFull;
        st.push(rx_frame{v - 1, op.arg4, pc + 1});
        pc = op.arg4;
      }
      break;
    default: ++pc; break;
    }
  }
}

// The plan of a record index, for the segment and emit kernels.  fpc /
// fd: the first op whose word is checked (a length, count, discriminant or
// validated enum) and its byte offset in the record -- every op before it
// has a fixed size -- or fpc = RX_BAD.  Its check is a necessary condition
// for a word to start a record: the segment kernel loads that word for all
// of a thread's candidate starts at once and walks only the ones that pass.
struct rx_plan {
  const xdrg_op *ops;
  const uint32_t *table;
  uint32_t nops;
  uint32_t fpc, fd;
};

__device__ __forceinline__ bool rx_first_ok(const xdrg_op &op, const uint32_t *__restrict__ table,
                                            uint32_t v) {
  switch (op.kind) {
  case XDRG_OP_ENUM: return enum_ok(table, op.arg0, op.arg1, v);
  case XDRG_OP_UNION:
    return (!(op.flags & XDRG_F_VALIDATE) || enum_ok(table, op.arg0, op.arg1, v)) &&
           union_target(op, table, v) >= 0;
  default: return v <= op.arg0;  // VAROPAQUE, STRING, VECTOR
  }
}

// The interpreted parse of a record start (rx_len over the plan's ops in
// dynamic LDS) for ix_seg_body (index_kernels.h).
struct rx_interp {
  rx_plan rp;
  __device__ __forceinline__ void init(uint32_t *smem) const {
    load_ops(reinterpret_cast<xdrg_op *>(smem), rp.ops, rp.nops);
  }
  __device__ __forceinline__ bool first_ok(const uint32_t *smem, uint32_t v) const {
    return rx_first_ok(reinterpret_cast<const xdrg_op *>(smem)[rp.fpc], rp.table, v);
  }
  __device__ __forceinline__ uint64_t first_len(uint32_t) const { return 0; }  // (no second filter)
  __device__ __forceinline__ bool second_ok(uint32_t, uint32_t) const { return true; }
  __device__ __forceinline__ uint32_t rlen(const uint32_t *smem, const uint8_t *s, uint64_t len, uint64_t a,
                                           uint32_t maxlen) const {
    return rx_len(reinterpret_cast<const xdrg_op *>(smem), rp.table, rx_global{s}, len, a, maxlen);
  }
};

// skip (record index): 1 when the fast path (rxs_*) holds the index; the
// list ranking's kernels then return at once.
__device__ __forceinline__ bool ix_skip(const uint32_t *skip) { return skip && *skip == 1u; }

template <bool REC>
__global__ __launch_bounds__(256) void k_ix_seg(const uint8_t *__restrict__ s, uint64_t len,
                                                uint32_t maxlen, uint32_t K,
                                                uint64_t *__restrict__ tab,
                                                uint32_t *__restrict__ list,
                                                uint32_t *__restrict__ lcount, rx_plan rp,
                                                const uint32_t *__restrict__ skip) {
  if (ix_skip(skip)) return;
  ix_seg_body<REC>(rx_interp{rp}, s, len, maxlen, K, tab, list, lcount, rp.fpc != RX_BAD, rp.fd);
}

// The fast path's scan-side kernels (index_kernels.h); its walk is the
// plan's generated xdrg_spec_rxs_walk.
template <bool LONG>
__global__ __launch_bounds__(256) void k_rxs_check(uint64_t *__restrict__ seg, const uint16_t *__restrict__ nodes,
                                                   uint64_t nseg, uint64_t len, unsigned long long *__restrict__ cnt,
                                                   uint32_t *__restrict__ flag, uint64_t *__restrict__ list,
                                                   unsigned long long *nl) {
  rxs_check_body<LONG>(seg, nodes, nseg, len, cnt, flag, list, nl);
}
template <bool EXACT>
__global__ __launch_bounds__(256) void k_rxs_emit(const uint64_t *__restrict__ seg,
                                                  const uint16_t *__restrict__ nodes,
                                                  const unsigned long long *__restrict__ base,
                                                  const xdrg_status *__restrict__ tot, uint64_t len, uint64_t n,
                                                  uint64_t *__restrict__ offsets, uint64_t *__restrict__ count,
                                                  uint32_t *__restrict__ flag, uint64_t nseg, uint32_t *hflag,
                                                  const unsigned long long *__restrict__ cnt) {
  rxs_emit_body<EXACT>(seg, nodes, base, tot, len, n, offsets, count, flag, nseg, hflag, cnt);
}
// The walk over a message stream's record marks (xdrg_index_msgs).
__global__ __launch_bounds__(64) void k_rxs_walk_msgs(const uint8_t *__restrict__ s, uint64_t len,
                                                      uint32_t maxlen, uint64_t *__restrict__ seg,
                                                      uint16_t *__restrict__ nodes, uint32_t *__restrict__ flag) {
  rxs_walk_body(mark_rx{maxlen}, s, len, maxlen, seg, nodes, flag, true, 0u);
}

// One node of the next level per workgroup: F children composed for
// every entry.  Also writes each child's inclusive prefix composition
// (pf: the group's first child up to this one, from every entry), so that
// the down pass hands every child its entry with one lookup.  out may be
// null (the top level needs only the prefixes).  LDS: the children's
// tables staged first.
template <bool LDS>
__global__ __launch_bounds__(256) void k_ix_up(const uint64_t *__restrict__ in, uint64_t nin,
                                               uint32_t K, uint32_t F, uint64_t *__restrict__ out,
                                               uint64_t *__restrict__ pf, const uint32_t *__restrict__ skip) {
  extern __shared__ __attribute__((aligned(16))) uint64_t stg[];
  if (ix_skip(skip)) return;
  const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * F;
  const uint32_t nc = static_cast<uint32_t>(min<uint64_t>(F, nin - c0));
  const uint64_t *src = in + c0 * K;
  uint64_t *pre = pf + c0 * K;
  if (LDS) {
    for (uint32_t i = threadIdx.x; i < nc * K; i += 256) stg[i] = src[i];
    __syncthreads();
  }
  for (uint32_t e = threadIdx.x; e < K; e += 256) {
    uint64_t x = e, c = 0, res = 0;
    bool term = false;
    for (uint32_t j = 0; j < nc; ++j) {
      if (!term) {
        const uint64_t t = LDS ? stg[j * K + x] : src[static_cast<uint64_t>(j) * K + x];
        c += t & kIxCnt;
        if (t >> 56) { res = (t >> 56) << 56 | c; term = true; }
        else x = (t >> 40) & 0xffffu;
      }
      pre[static_cast<uint64_t>(j) * K + e] = term ? res : (x << 40 | c);
    }
    if (out) out[static_cast<uint64_t>(blockIdx.x) * K + e] = term ? res : (x << 40 | c);
  }
}

// Entry word of a node: bit 63 = off the chain; entry << 40; messages
// before the node (40 bits).  One workgroup per parent, one thread per
// child: the child's entry is the parent's through the prefix composition
// of the children before it (k_ix_up's pf).
__global__ __launch_bounds__(64) void k_ix_down(const uint64_t *__restrict__ pf, uint64_t nin,
                                                uint32_t K, uint32_t F,
                                                const uint64_t *__restrict__ up,
                                                uint64_t *__restrict__ ent, const uint32_t *__restrict__ skip) {
  if (ix_skip(skip)) return;
  const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * F;
  const uint32_t nc = static_cast<uint32_t>(min<uint64_t>(F, nin - c0));
  const uint32_t j = threadIdx.x;
  if (j >= nc) return;
  const uint64_t e = up[blockIdx.x];
  if (e >> 63) {
    ent[c0 + j] = 1ull << 63;
    return;
  }
  const uint64_t x = (e >> 40) & 0xffffu, b = e & kIxCnt;
  if (j == 0) {
    ent[c0] = x << 40 | b;
    return;
  }
  const uint64_t t = pf[(c0 + j - 1) * K + x];
  ent[c0 + j] = (t >> 56) ? (1ull << 63) : (((t >> 40) & 0xffffu) << 40 | (b + (t & kIxCnt)));
}

// Segments on the chain.  The nodes reachable from the entry x are found by
// doubling over the segment's valid-node list (Reach_{k+1} = Reach_k plus
// the 2^k-th successors of Reach_k); since positions grow along the chain,
// a node's message index is b + (reachable nodes before it).  The node
// where the chain ends (the last reachable one, unless the chain leaves the
// segment) is classified exactly as read_message would (ix_mark).
// REC: the chain of records ends at w: the end of the stream, or a record
// that does not parse (its decode reports why) -- or one longer than the
// index window, XDRG_ERR_INDEX_LONG.
// A message index over a window of a longer stream (xdrg_index_msgs with a
// max_msg_len past XDRG_INDEX_MAX_MSG, ix_window below): the window's
// place in the stream, and where the chain leaves it.  For any other index
// m0 = base = 0, next = nullptr and the window is the stream.
struct ix_cont {
  uint64_t m0;               // messages before the window
  uint64_t base;             // byte offset of the window in the stream
  const uint8_t *s;          // the whole stream
  uint64_t len;              // its length
  uint32_t maxlen;           // the caller's max_msg_len
  unsigned long long *next;  // the chain leaves at: [mark word, message index]
};

template <bool REC>
__device__ void ix_final(const uint8_t *__restrict__ s, uint64_t len, uint32_t maxlen, uint64_t w,
                         uint64_t m, uint64_t max_msgs, uint64_t *__restrict__ offsets,
                         unsigned long long *count, unsigned long long *err, const rx_plan &rp,
                         const ix_cont &C) {
  if (m > max_msgs) return;
  offsets[m] = C.base + 4 * w;
  if (REC) {
    if (C.next) {
      // a window of a longer stream (rx_windows): a record that parses in
      // the whole stream -- longer than the window, nested deeper than its
      // frames, or past the window's end -- is where the next round picks up
      // (record n too: whether one parses after the n-th decides the count)
      const uint64_t aw = C.base / 4 + w;
      if (4 * aw < C.len && rx_len(rp.ops, rp.table, rx_global{C.s}, C.len, 4 * aw, maxlen) != RX_BAD) {
        C.next[0] = aw;
        C.next[1] = C.m0 + m;
        return;
      }
    } else if (4 * w < len && m < max_msgs &&
               rx_len(rp.ops, rp.table, rx_global{s}, len, 4 * w, maxlen) == RX_LONG) {
      report(err, m, kOpRecordLevel, XDRG_ERR_INDEX_LONG);
    }
  } else {
    uint64_t nx = 0;
    uint32_t st = ix_mark(4 * w + 4 <= len ? ld32(s + 4 * w) : 0u, w, len, maxlen, &nx);
    if (C.next && !(st == IX_END && C.base + len == C.len)) {
      // a mark the window cannot hold (a longer message, or one past the
      // window's end), or the window's end: the chain goes on there unless
      // the stream itself says otherwise (classified as read_message would)
      const uint64_t aw = C.base / 4 + w;
      const uint32_t rs = ix_mark(4 * aw + 4 <= C.len ? ld32(C.s + 4 * aw) : 0u, aw, C.len, C.maxlen, &nx);
      if (m < max_msgs && (rs == IX_RUN || st == IX_END)) {
        C.next[0] = aw;
        C.next[1] = C.m0 + m;
        return;
      }
      st = m == max_msgs ? IX_LONG : rs;  // the capacity (MSG_COUNT below), or what the stream says
    }
    if (st != IX_END) report(err, C.m0 + m, kOpRecordLevel, m == max_msgs ? XDRG_ERR_MSG_COUNT : ix_error(st));
  }
  atomicMin(count, C.m0 + m);
}

template <bool REC>
__global__ __launch_bounds__(256) void k_ix_emit(const uint8_t *__restrict__ s, uint64_t len,
                                                 uint32_t maxlen, const uint64_t *__restrict__ ent,
                                                 const uint32_t *__restrict__ list,
                                                 const uint32_t *__restrict__ lcount,
                                                 uint64_t *__restrict__ offsets, uint64_t max_msgs,
                                                 unsigned long long *count,
                                                 unsigned long long *err, rx_plan rp, ix_cont C,
                                                 const uint32_t *__restrict__ skip) {
  if (ix_skip(skip)) return;
  // J: successor of a valid node (0xffff: not a valid node); lst: the valid
  // nodes; nj / mk: a round's new successors and marks (double buffer)
  __shared__ __attribute__((aligned(16))) uint16_t J[kIxSW];
  __shared__ uint16_t lst[kIxSW], nj[kIxSW], mk[kIxSW];
  __shared__ __attribute__((aligned(16))) uint8_t on[kIxSW];  // reachable from the entry
  __shared__ uint32_t seen[kIxSW / 32];                       // successor of a node >= x
  __shared__ uint32_t wtot[4];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  // the entry, the list length and the list's first 256 words in one round trip
  const uint32_t *gl = list + static_cast<uint64_t>(blockIdx.x) * kIxSW;
  const uint64_t e = ent[blockIdx.x];
  const uint32_t nvalid = lcount[blockIdx.x];
  const uint32_t v0 = gl[tid];  // inside the workspace; used only when tid < nvalid
  if (e >> 63) return;
  const uint64_t b = e & kIxCnt;
  if (b > max_msgs) return;  // past the index's capacity: reported where it ran out
  const uint32_t x = static_cast<uint32_t>((e >> 40) & 0xffffu);
  const uint64_t w0 = static_cast<uint64_t>(blockIdx.x) * kIxSW;
  const u32x4 ones = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  reinterpret_cast<u32x4 *>(J)[tid] = ones;
  reinterpret_cast<u32x4 *>(J)[tid + 256] = ones;
  reinterpret_cast<u32x4 *>(on)[tid] = u32x4{0, 0, 0, 0};
  if (tid < kIxSW / 32) seen[tid] = 0;
  __syncthreads();
  for (uint32_t j = tid; j < nvalid; j += 256) {
    const uint32_t v = j == tid ? v0 : gl[j];
    J[v & 0xfffu] = static_cast<uint16_t>(v >> 12);
    lst[j] = static_cast<uint16_t>(v & 0xfffu);
  }
  if (tid == 0) on[x] = 1;
  __syncthreads();
  if (J[x] == 0xffffu) {  // the chain ends at its entry
    if (tid == 0) ix_final<REC>(s, len, maxlen, w0 + x, b, max_msgs, offsets, count, err, rp, C);
    return;
  }
  // Fast path: when the valid nodes from x on form one path (no node is the
  // successor of two of them and each but x is the successor of one), the
  // chain is exactly those nodes plus the word where it ends; true unless
  // message bodies hold words that read as marks.
  bool slow = false;
  for (uint32_t j = tid; j < nvalid; j += 256) {
    const uint32_t i = lst[j];
    if (i < x) continue;
    on[i] = 1;
    const uint32_t t = J[i];
    if (t < kIxSW) {
      const uint32_t bit = 1u << (t & 31u);
      if (atomicOr(&seen[t >> 5], bit) & bit) slow = true;  // two predecessors
      if (J[t] == 0xffffu) on[t] = 1;                        // the chain ends at t
    }
  }
  slow = __syncthreads_or(slow);
  if (!slow) {
    for (uint32_t j = tid; j < nvalid; j += 256) {
      const uint32_t i = lst[j];
      if (i > x && !(seen[i >> 5] & (1u << (i & 31u)))) slow = true;  // a second path
    }
    slow = __syncthreads_or(slow);
  }
  if (slow) {
    reinterpret_cast<u32x4 *>(on)[tid] = u32x4{0, 0, 0, 0};
    __syncthreads();
    if (tid == 0) on[x] = 1;
    __syncthreads();
  }
  // slow path, doubling: read phase into nj / mk, barrier, write phase (Jacobi)
  for (uint32_t k = 0; slow && k < 2 * kIxLog + 2; ++k) {
    for (uint32_t j = tid; j < nvalid; j += 256) {
      const uint32_t i = lst[j];
      const uint32_t ji = J[i];
      const uint32_t jj = ji < kIxSW ? J[ji] : 0xffffu;
      nj[j] = static_cast<uint16_t>(jj != 0xffffu ? jj : ji);
      mk[j] = static_cast<uint16_t>(on[i] && ji < kIxSW ? ji : 0xffffu);
    }
    __syncthreads();
    bool changed = false;
    for (uint32_t j = tid; j < nvalid; j += 256) {
      const uint32_t i = lst[j], m = mk[j], v = nj[j];
      if (m != 0xffffu && !on[m]) { on[m] = 1; changed = true; }
      if (v != J[i]) { J[i] = static_cast<uint16_t>(v); changed = true; }
    }
    if (!__syncthreads_or(changed)) break;
  }
  // rank the reachable nodes by position: thread t owns nodes [16t, 16t + 16)
  const u32x4 f = reinterpret_cast<const u32x4 *>(on)[tid];
  const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
  uint32_t cnt = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) cnt += __popc(fw[q] & 0x01010101u);
  uint32_t incl = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= static_cast<uint32_t>(o)) incl += y;
  }
  if (lane == 63) wtot[wid] = incl;
  __syncthreads();
  uint32_t r = incl - cnt, total = 0;
  for (uint32_t w = 0; w < 4; ++w) {
    if (w < wid) r += wtot[w];
    total += wtot[w];
  }
  for (uint32_t q = 0; q < 16; ++q) {
    if (!((fw[q >> 2] >> (8 * (q & 3))) & 1u)) continue;
    const uint32_t i = 16u * tid + q;
    const uint64_t m = b + r;
    ++r;
    if (r == total && J[i] == 0xffffu) {  // the chain ends at this node
      ix_final<REC>(s, len, maxlen, w0 + i, m, max_msgs, offsets, count, err, rp, C);
      continue;
    }
    if (m > max_msgs) continue;
    offsets[m] = C.base + 4 * (w0 + i);
    if (m == max_msgs && !REC) {  // a message past the index's capacity
      report(err, C.m0 + m, kOpRecordLevel, XDRG_ERR_MSG_COUNT);
      atomicMin(count, C.m0 + m);
    }
  }
}

// Records after the one where the chain ended: [len, len).
__global__ void k_rx_fill(uint64_t *__restrict__ offsets, const unsigned long long *__restrict__ count,
                          uint64_t n, uint64_t len, const uint32_t *__restrict__ skip) {
  if (ix_skip(skip)) return;
  const uint64_t c = *count;  // all-ones: the chain went past record n
  if (c >= n) return;
  for (uint64_t i = c + 1 + static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i <= n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    offsets[i] = len;
}

// Messages longer than one index window, walked mark after mark as
// read_message frames them (srpc.cc:29-55): from next = [mark word,
// message index] while the message there is longer than
// XDRG_INDEX_MAX_MSG, at most `hops` of them.  Leaves next at the first
// shorter message (next[2] = 1) or at the hop budget (next[2] = 0); the
// end of the stream, a framing error or the index's capacity ends the
// index here (next[0] = all ones).
__global__ void k_ix_long(const uint8_t *__restrict__ s, uint64_t len, uint32_t maxlen, uint64_t max_msgs,
                          uint64_t *__restrict__ offsets, unsigned long long *count, unsigned long long *err,
                          unsigned long long *next, uint32_t hops) {
  if (threadIdx.x || blockIdx.x) return;
  uint64_t w = next[0], m = next[1];
  for (uint32_t h = 0; h < hops; ++h) {
    uint64_t nx = 0;
    const uint32_t st = ix_mark(4 * w + 4 <= len ? ld32(s + 4 * w) : 0u, w, len, maxlen, &nx);
    if (st == IX_RUN && 4 * (nx - w - 1) <= XDRG_INDEX_MAX_MSG) {  // a window takes it
      next[0] = w;
      next[1] = m;
      next[2] = 1;
      return;
    }
    if (m > max_msgs) break;  // not reached: the capacity is checked below
    offsets[m] = 4 * w;
    if (st != IX_RUN || m == max_msgs) {
      if (st != IX_END) report(err, m, kOpRecordLevel, m == max_msgs ? XDRG_ERR_MSG_COUNT : ix_error(st));
      atomicMin(count, m);
      next[0] = ~0ull;
      return;
    }
    ++m;
    w = nx;
  }
  next[0] = w;
  next[1] = m;
  next[2] = 0;
}

// k_rx_long's stream reader.  The wave's 64 lanes parse the same record in
// step (the same values in every lane), through a 4 KiB block of the stream
// in LDS: a word outside it reloads the block, each lane loading four
// 16-byte chunks, so one round trip brings 4 KiB where a lone lane's parse
// waited on every length and count (rp_list's 500-node lists: 64 ms for
// the index of 1M records, profiles/r05k).  Positions are word-aligned
// record offsets, and a word is read only when it lies inside the stream.
struct rx_wave_cache {
  const uint8_t *s;
  uint64_t len;
  uint32_t *buf;          // 1024 words of LDS
  mutable uint64_t base;  // stream offset of buf[0] (4 KiB aligned; ~0: none)
  __device__ __forceinline__ uint32_t operator()(uint64_t p) const {
    if (p < base || p - base >= 4096u) {
      const uint64_t b = p & ~4095ull;
      wave_sync();  // every lane past its reads of the old block
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t k = threadIdx.x + 64u * j;
        const uint64_t o = b + 16ull * k;
        u32x4 v{0u, 0u, 0u, 0u};
        if (o + 16 <= len) {
          v = ld16u(s + o);
        } else if (o < len) {
          v.x = partial_word(s, len, o);
          v.y = partial_word(s, len, o + 4);
          v.z = partial_word(s, len, o + 8);
          v.w = partial_word(s, len, o + 12);
        }
        *reinterpret_cast<u32x4 *>(buf + 4u * k) = v;
      }
      wave_sync();
      base = b;
    }
    return buf[(p - base) >> 2];
  }
};

// Records too long for an index window (or nested deeper than its frames),
// walked one after another from next = [word, record index] as
// xdr_from_opaque's own walk would (marshal.h:299-306): while the record
// there is such a record, at most `hops` of them, each parsed whole
// (lengths, counts and discriminants; its frames in registers, or in `slab`
// past XDRG_INDEX_FRAMES).  Leaves next at the first record a window takes
// (next[2] = 1) or at the hop budget (next[2] = 0); the end of the stream,
// the n-th record or a record that does not parse ends the index here
// (next[0] = all ones; the record it stops at gets its offset, k_rx_fill
// the rest).  One wave, every lane on the same parse (rx_wave_cache); lane
// 0 writes.
__global__ __launch_bounds__(64) void k_rx_long(const uint8_t *__restrict__ s, uint64_t len, uint32_t maxlen,
                                                uint64_t n, const xdrg_op *__restrict__ ops,
                                                const uint32_t *__restrict__ table, uint64_t *__restrict__ offsets,
                                                unsigned long long *count, unsigned long long *next, rx_frame *slab,
                                                uint32_t hops, uint32_t nops, uint32_t ops_lds) {
  __shared__ __attribute__((aligned(16))) uint32_t cbuf[1024];
  extern __shared__ __attribute__((aligned(16))) uint32_t rsm[];  // the plan's ops (ops_lds)
  if (blockIdx.x) return;
  if (ops_lds) {  // each op dispatch a round trip to L2 otherwise
    load_ops(reinterpret_cast<xdrg_op *>(rsm), ops, nops);
    ops = reinterpret_cast<const xdrg_op *>(rsm);
  }
  const bool l0 = threadIdx.x == 0;
  const rx_wave_cache rd{s, len, cbuf, ~0ull};
  uint64_t w = next[0], m = next[1];
  for (uint32_t h = 0; h < hops; ++h) {
    if (4 * w >= len) {  // the stream's end
      if (l0) {
        offsets[m] = len;
        atomicMin(count, m);
        next[0] = ~0ull;
      }
      return;
    }
    // the whole record: in registers, or (nested past them) in the slab
    uint32_t L = rx_len<rx_wave_cache, uint64_t, rx_reg_frames, true>(ops, table, rd, len, 4 * w, 0xffffffffu);
    const bool deep = L == RX_LONG;
    if (deep)
      L = rx_len<rx_wave_cache, uint64_t, rx_slab_frames, true>(ops, table, rd, len, 4 * w, 0xffffffffu,
                                                                rx_slab_frames{slab, XDRG_MAX_FRAMES, 0});
    if (m >= n) {  // n records and more bytes (the decode reports them): the
      // count stays all ones if a record parses there (the chain goes on)
      if (l0) {
        offsets[n] = 4 * w;
        if (L == RX_BAD || L == RX_LONG) atomicMin(count, n);
        next[0] = ~0ull;
      }
      return;
    }
    if (!deep && L != RX_BAD && L <= maxlen && rx_len(ops, table, rd, len, 4 * w, maxlen) != RX_LONG) {
      // a window takes it (its parse, frames counted, does not call it long)
      if (l0) {
        next[0] = w;
        next[1] = m;
        next[2] = 1;
      }
      return;
    }
    if (l0) offsets[m] = 4 * w;
    if (L == RX_BAD || L == RX_LONG) {  // a record the decode rejects
      if (l0) {
        atomicMin(count, m);
        next[0] = ~0ull;
      }
      return;
    }
    ++m;
    w += L / 4;
  }
  if (l0) {
    next[0] = w;
    next[1] = m;
    next[2] = 0;
  }
}

// xdrg_encode_sizes of a fixed plan: the total is known.
__global__ void k_set_total(xdrg_status *st, uint64_t v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) st->total_bytes = v;
}

// ------------------------------------------------------------------ swaps
__global__ void k_swap32(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint64_t n) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = bswap32(in[i]);
}
__global__ void k_swap64(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = __builtin_bswap64(in[i]);
}

// ------------------------------------------------------------------ host
constexpr uint64_t kMallBytes = 256ull << 20;  // MI355X Infinity Cache
constexpr uint32_t kVarLdsBudget = 64u << 10;  // wave-cooperative var kernels
uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
bool aligned(const void *p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }
uint32_t gcd32(uint32_t a, uint32_t b) { while (b) { uint32_t t = a % b; a = b; b = t; } return a; }

// Fixed plans: first op whose wire bytes do not fit in `rem` bytes.
uint32_t first_op_past(const xdrg_plan &p, uint64_t rem) {
  for (uint32_t i = 0; i + 1 < p.ops.size(); ++i) {
    const xdrg_op &op = p.ops[i];
    const uint64_t sz = op.kind == XDRG_OP_U64 ? 8 : op.kind == XDRG_OP_OPAQUE ? op.arg0 : 4;
    if (p.op_wire_off[i] + sz > rem) return i;
  }
  return 0;
}
uint32_t first_op_deeper(const xdrg_plan &p, uint32_t limit) {
  for (uint32_t i = 0; i < p.ops.size(); ++i)
    if (p.ops[i].kind != XDRG_OP_END && p.ops[i].kind != XDRG_OP_JUMP && p.ops[i].depth > limit)
      return i;
  return 0;
}

int launch_report(unsigned long long *err, uint64_t rec, uint32_t op, uint32_t code,
                  hipStream_t s) {
  k_report<<<1, 64, 0, s>>>(err, rec, op, code);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

// Runs one fixed program (encode or decode) over nrec records.
int run_fixed(const xdrg_plan &p, const dev_tables &T, bool decode, const void *in, void *out,
              uint64_t nrec, unsigned long long *err, hipStream_t s) {
  const plan_opts &O = p.opts;
  if (nrec == 0) return XDRG_OK;
  const fixed_prog &pg = decode ? p.dec : p.enc;
  const bool checks = decode && p.has_checks;
  if (p.path == XDRG_PATH_FIXED_REG && aligned(in, 16) && aligned(out, 16)) {
    // Launch shapes from tools/tune/tune_fixed.py (rec128) and the copy
    // ceiling probe (tools/probe/copy_ceiling.hip, profiles/r03c):
    //  * working set (input + output) that fits the 256 MiB Infinity Cache
    //    (1M records = 256 MiB): plain 16-byte loads/stores, one chunk in
    //    flight per lane, 1024 workgroups -> 6.9 TB/s back to back;
    //  * past the cache, up to 1 GiB in+out (config 5's 2M-record shard per
    //    rank is 512 MiB): the same 1024-workgroup loop with non-temporal
    //    loads and stores, 5.85-6.10 TB/s at 384-768 MiB against 5.55-5.71
    //    for the plain loop and 5.60-5.83 for the one-shot grid
    //    (tools/gpu/fixed_shape_sweep.py, profiles/r06_fixed);
    //  * larger batches stream from HBM: one chunk per lane over a one-shot
    //    grid with non-temporal loads and stores -- the box's best 16-byte
    //    copy past the cache, 6.58 TB/s at 2 GiB per buffer, where any
    //    grid-stride loop measured 4.6-5.6 TB/s (the old 512-workgroup,
    //    two-in-flight shape: 5.54 TB/s at 16M records).
    const uint32_t W = p.fixed_size;
    const uint32_t cpr = W / 16;
    const uint64_t nchunks = nrec * cpr;
    const uint64_t ws_bytes = nchunks * 32ull;  // in + out
    // XDRG_OPT_FIXED_STREAM picks the shape for A/B runs (bench.py shard_2m)
    const int fs = O.fixed_stream;
    const bool streaming = fs < 0 ? ws_bytes > kMallBytes : (fs == 1 || fs == 3);      // non-temporal accesses
    const bool one_shot = fs < 0 ? ws_bytes > 4 * kMallBytes : (fs == 1 || fs == 2);   // one chunk per lane
    uint64_t blocks = (nchunks + 255) / 256;
    if (!one_shot) blocks = std::min<uint64_t>(blocks, 1024);
    if (blocks > 0x7fffffffull) return XDRG_EUNSUPPORTED;
    const uint32_t g0 = cpr / gcd32(cpr, 256);
    blocks = align_up(std::max<uint64_t>(blocks, 1), g0);
    const reg_word *prog = decode ? T.d_dec_reg : T.d_enc_reg;
    const bool bools = pg.has_bool;
    const u32x4 *i4 = static_cast<const u32x4 *>(in);
    u32x4 *o4 = static_cast<u32x4 *>(out);
#define LAUNCH_REG(B, C)                                                                         \
  do {                                                                                           \
    if (streaming)                                                                               \
      k_fixed_reg<B, C, 1, true><<<blocks, 256, 0, s>>>(i4, o4, nchunks, cpr, prog, T.d_table, err); \
    else                                                                                         \
      k_fixed_reg<B, C, 1, false><<<blocks, 256, 0, s>>>(i4, o4, nchunks, cpr, prog, T.d_table, err); \
  } while (0)
    if (!bools && !checks) LAUNCH_REG(false, false);
    else if (bools && !checks) LAUNCH_REG(true, false);
    else if (!bools && checks) LAUNCH_REG(false, true);
    else LAUNCH_REG(true, true);
#undef LAUNCH_REG
    HIPCHK(hipGetLastError());
    return XDRG_OK;
  }
  if (!aligned(in, 4) || !aligned(out, 4)) return XDRG_EALIGN;
  // Tile path (kernels.h k_fixed_tile): records of up to 16 words each way,
  // up to 2 terms per output word, no decode checks.  numerics 1M: 16.5 us
  // vs the group kernel's 19.5 (profiles/r05l, r05m; FIXED_PATH 3 runs it).
  if (!checks && O.fixed_path == 0 && aligned(in, 16) && aligned(out, 16) && pg.in_words <= 16 &&
      pg.out_words <= 16 && pg.in_words && pg.out_words) {
    uint32_t kt = 0;
    for (const term_idx &ix : pg.idx) kt = std::max<uint32_t>(kt, ix.count);
    auto go = [&](auto tp) -> int {
      for (uint32_t j = 0; j < pg.out_words; ++j) {
        const term_idx ix = pg.idx[j];
        tp.nterm[j] = ix.count;
        for (uint32_t k = 0; k < ix.count; ++k) {
          const term &t = pg.terms[ix.start + k];
          tp.src[j][k] = t.src;
          tp.sel[j][k] = t.kind == T_BOOL ? (kGrpBool | t.sel) : t.sel;
        }
      }
      const uint64_t ntiles = (nrec + kTileRec - 1) / kTileRec;
      constexpr int KT = sizeof(tp.src[0]) / sizeof(uint32_t);
      const size_t lds = 4ull * (kTileRec * (pg.in_words + pg.out_words) + 4);
      // one workgroup per resident slot: numerics 1M (25.6 KiB of LDS, 6 per
      // CU) 16.5 us at 1536 workgroups, 18.4 at 1024, 18.6 at 2048, 22.0 at
      // 512 (profiles/r05m)
      // (the query's answer cached per device, term count and LDS size: it
      // cost host time on every call of a 16 us kernel)
      uint64_t resident = 1024;
      {
        struct occ_key { int dev, kt; size_t lds; uint64_t resident; };
        static std::mutex mu;
        static std::vector<occ_key> seen;
        int dev = 0;
        bool hit = false;
        if (hipGetDevice(&dev) == hipSuccess) {
          {
            std::lock_guard<std::mutex> g(mu);
            for (const occ_key &k : seen)
              if (k.dev == dev && k.kt == KT && k.lds == lds) { resident = k.resident; hit = true; break; }
          }
          int cus = 0, occ = 0;
          if (!hit && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
              hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fixed_tile<16, 16, KT>, 256, lds) == hipSuccess &&
              cus > 0 && occ > 0) {
            resident = uint64_t(cus) * uint64_t(occ);
            std::lock_guard<std::mutex> g(mu);
            seen.push_back(occ_key{dev, KT, lds, resident});
          }
        }
      }
      const uint64_t blocks = std::min<uint64_t>(ntiles, O.grp_blocks ? uint64_t(O.grp_blocks) : resident);
      k_fixed_tile<16, 16, KT><<<static_cast<uint32_t>(blocks), 256, lds, s>>>(
          static_cast<const u32x4 *>(in), static_cast<u32x4 *>(out), nrec, pg.in_words, pg.out_words, tp);
      HIPCHK(hipGetLastError());
      return XDRG_OK;
    };
    if (kt == 1) return go(tile_prog<16, 1>{});
    if (kt == 2) return go(tile_prog<16, 2>{});
  }
  if (pg.grp_G && !checks && O.fixed_path != 2 && aligned(in, 16) && aligned(out, 16) &&
      nrec >= pg.grp_G) {
    // Group path over the full groups; the tail (< G records) below.
    const uint64_t ngroups = nrec / pg.grp_G;
    const uint64_t nchunks = ngroups * pg.grp_C;
    const uint32_t in_g = pg.grp_G * pg.in_words * 4u;
    const uint64_t cap = O.grp_blocks ? uint64_t(O.grp_blocks) : 2048u;
    uint64_t blocks = std::min<uint64_t>((nchunks + 255) / 256, cap);
    blocks = align_up(std::max<uint64_t>(blocks, 1), pg.grp_C / gcd32(pg.grp_C, 256));
    const grp_term *prog = decode ? T.d_dec_grp : T.d_enc_grp;
    const uint8_t *i8 = static_cast<const uint8_t *>(in);
    u32x4 *o4 = static_cast<u32x4 *>(out);
    // tools/tune/tune_grp.py (numerics 1M): U=4 / 2048 workgroups best, within 10 %
    const int U = O.grp_unroll ? O.grp_unroll : (pg.grp_KT == 1 ? 4 : pg.grp_KT == 2 ? 2 : 1);
#define LAUNCH_GRP(KT, UU)                                                                   \
  do {                                                                                       \
    if (O.grp_nontemporal)                                                                            \
      k_fixed_grp<KT, UU, true><<<blocks, 256, 0, s>>>(i8, o4, nchunks, pg.grp_C, in_g, prog); \
    else                                                                                     \
      k_fixed_grp<KT, UU, false><<<blocks, 256, 0, s>>>(i8, o4, nchunks, pg.grp_C, in_g, prog); \
  } while (0)
    if (pg.grp_KT == 1) {
      if (U == 1) LAUNCH_GRP(1, 1); else if (U == 2) LAUNCH_GRP(1, 2); else LAUNCH_GRP(1, 4);
    } else if (pg.grp_KT == 2) {
      if (U == 1) LAUNCH_GRP(2, 1); else LAUNCH_GRP(2, 2);
    } else {
      LAUNCH_GRP(4, 1);
    }
#undef LAUNCH_GRP
    HIPCHK(hipGetLastError());
    const uint64_t done = ngroups * pg.grp_G;
    if (done == nrec) return XDRG_OK;
    in = static_cast<const uint8_t *>(in) + done * pg.in_words * 4u;
    out = static_cast<uint8_t *>(out) + done * pg.out_words * 4u;
    nrec -= done;
  }
  const uint32_t in_words = pg.in_words, out_words = pg.out_words;
  if (in_words > 8192) return XDRG_EUNSUPPORTED;  // > 32 KiB records: tile won't fit
  uint32_t TR = std::min<uint32_t>(256, std::max<uint32_t>(4, 8192 / in_words));
  TR &= ~3u;
  const bool vec = aligned(in, 16) && aligned(out, 16) && (TR * in_words) % 4 == 0 &&
                   (TR * out_words) % 4 == 0;
  const size_t lds = 4ull * (TR * in_words + 4) + 4ull * ((out_words + 3u) & ~3u) +
                     sizeof(term) * pg.terms.size();
  const uint64_t tiles = (nrec + TR - 1) / TR;
  const uint64_t blocks = std::min<uint64_t>(tiles, 4096);
  const term_idx *idx = decode ? T.d_dec_idx : T.d_enc_idx;
  const term *terms = decode ? T.d_dec_terms : T.d_enc_terms;
  const uint32_t nterms = uint32_t(pg.terms.size());
  const uint32_t nchecks = checks ? uint32_t(p.checks.size()) : 0u;
  auto *i32 = static_cast<const uint32_t *>(in);
  auto *o32 = static_cast<uint32_t *>(out);
#define LAUNCH_LDS(C, V)                                                                   \
  k_fixed_lds<C, V><<<blocks, 256, lds, s>>>(i32, o32, nrec, in_words, out_words, TR, idx, \
                                             terms, nterms, T.d_checks, nchecks, T.d_table, err)
  if (checks) {
    if (vec) LAUNCH_LDS(true, true); else LAUNCH_LDS(true, false);
  } else {
    if (vec) LAUNCH_LDS(false, true); else LAUNCH_LDS(false, false);
  }
#undef LAUNCH_LDS
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

// Var workspace: u32 sizes[n], the 64-record block sums, then their
// exclusive scan (a separate array: the multi-workgroup scan reads the sums
// while other workgroups write the bases).
size_t var_ws_layout(uint64_t n, size_t *sizes_off, size_t *bsum_off, size_t *base_off = nullptr) {
  const uint64_t nb = (n + 63) / 64;  // block sums at the finest block size (64)
  *sizes_off = 0;
  *bsum_off = align_up(n * 4, 256);
  const size_t b2 = *bsum_off + align_up((nb + 1) * 8, 256);
  if (base_off) *base_off = b2;
  return b2 + align_up((nb + 1) * 8, 256);
}

// Heap bytes xdrg_decode needs (include/xdrgpu.h xdrg_decode_heap_size).
uint64_t decode_heap_bytes(const xdrg_plan &p, uint64_t len) {
  return p.has_vector ? align_up(len, 16) + static_cast<uint64_t>(p.heap_factor) * len : len;
}

// Size pass (xdr_size per record + 64-record block sums).
// Size pass of a linear plan (xdrg_plan::linear): no walk.  One lane per
// record reads the length words of its bytes fields (independent loads);
// 256-record workgroups, one 64-record block sum per wave.
struct lin_args {
  uint32_t base, n;
  uint32_t off[8];
};
__global__ __launch_bounds__(256) void k_size_linear(const uint8_t *__restrict__ native, uint64_t n,
                                                     uint32_t stride, lin_args L,
                                                     uint32_t *__restrict__ sizes,
                                                     unsigned long long *__restrict__ block_sums,
                                                     uint32_t mark, unsigned long long *err) {
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  uint32_t size = 0;
  if (r < n) {
    const uint8_t *rec = native + r * stride;
    uint32_t len[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      len[k] = static_cast<uint32_t>(k) < L.n ? *reinterpret_cast<const uint32_t *>(rec + L.off[k] + 8) : 0u;
    uint64_t sz = static_cast<uint64_t>(L.base) + mark;
#pragma unroll
    for (int k = 0; k < 8; ++k) sz += (static_cast<uint64_t>(len[k]) + 3u) & ~3ull;
    if (sz >= kSizeErr) {
      report(err, r, 0, XDRG_ERR_OVERFLOW_PUT);
      size = kSizeErr;
    } else {
      size = static_cast<uint32_t>(sz);
    }
    sizes[r] = size;
  }
  unsigned long long v = (size & kSizeErr) ? 0ull : size;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const uint64_t blk = r / 64u;
  if (block_sums && (threadIdx.x & 63u) == 0 && blk * 64u < n) block_sums[blk] = v;
}

// ------------------------------------------------------------ deep passes
// The deep passes of the element-subroutine walks (sub_kernels.h) of a plan
// that can nest past XDRG_SUB_FRAMES (plan.deep): the lists of deferred
// records and the frame slabs of the two deep passes, in caller memory (the
// workspace, include/xdrgpu.h xdrg_deep_workspace_size): no allocation, no
// lock and no state shared between calls, so calls on different streams run
// side by side and graph capture records plain memsets and kernels.
constexpr uint32_t kDeepLanesA = 4096, kDeepSlabA = 1024;           // 96 MiB of frames (24 B each)
constexpr uint32_t kDeepLanesB = 8, kDeepSlabB = XDRG_MAX_FRAMES;   // 96 MiB
static_assert(kDeepLanesA % 256 == 0, "deep pass A runs 256-lane workgroups");
constexpr uint64_t kDeepSlabBytes =
    sizeof(sub_frame) * (uint64_t(kDeepLanesA) * kDeepSlabA + uint64_t(kDeepLanesB) * kDeepSlabB);

// The chain log (sub_kernels.h "Chains"): chains and logged nodes.
constexpr uint32_t kChainCap = 1u << 16, kNodeCap = 1u << 20;  // 24 MiB of nodes
constexpr uint32_t kChainGrid = 512;  // node pass workgroups (256 lanes, grid-stride over the nodes)
constexpr uint64_t kChainLogBytes = 8ull * kChainCap + sizeof(sub_node) * (uint64_t(kNodeCap) + kChainCap);

// [five counters | 256][list A: n u32][list B: n u32][slab A][slab B]
// [chain of each record: n u32][chain records, chain ends: kChainCap u32 each][nodes][chain heads]
// (The decode, which logs no chains, keeps its wave list -- sub_kernels.h
// "Long records" -- where the chain of each record goes.)
constexpr uint32_t kWaveGrid = 256;  // wave pass workgroups (kWaveWaves waves, a listed record per wave at a time)
uint64_t deep_area_bytes(const xdrg_plan &p, uint64_t n) {
  if (!p.deep) return 0;
  const uint64_t cap = std::max<uint64_t>(n, 1);
  return 256 + align_up(8 * cap, 256) + kDeepSlabBytes + align_up(4 * cap, 256) + kChainLogBytes;
}

struct deep_passes {
  sub_pass main{nullptr, nullptr, nullptr, nullptr, nullptr, 0, 1};
  sub_pass A{}, B{};
  bool on = false;  // the plan needs the deep passes
};

// The passes of plan p over n records on stream s, their memory at `area`
// (deep_area_bytes(p, n) bytes of the caller's workspace).
// reset = false: the lists a size pass over the same area left (the sized
// half of an encode, xdrg_encode_sized after xdrg_encode_sizes).
int deep_setup(const xdrg_plan &p, uint64_t n, void *area, size_t area_bytes, hipStream_t s, deep_passes &dp,
               bool reset = true) {
  if (!p.deep) return XDRG_OK;
  if (n > 0xffffffffull) return XDRG_EUNSUPPORTED;  // u32 list entries
  if (!area || area_bytes < deep_area_bytes(p, n) || !aligned(area, 256)) return XDRG_ESPACE;
  uint8_t *d = static_cast<uint8_t *>(area);
  // (the lists' and the log's counters, and the decode's wave list's)
  if (reset) HIPCHK(static_cast<hipError_t>(xdrg::fill32(d, 0u, 10, s)));
  auto *cnt = reinterpret_cast<unsigned long long *>(d);
  const uint64_t cap = std::max<uint64_t>(n, 1);
  uint32_t *la = reinterpret_cast<uint32_t *>(d + 256), *lb = la + cap;
  sub_frame *sa = reinterpret_cast<sub_frame *>(d + 256 + align_up(8 * cap, 256));
  sub_frame *sb = sa + uint64_t(kDeepLanesA) * kDeepSlabA;
  uint8_t *lg = d + 256 + align_up(8 * cap, 256) + kDeepSlabBytes;
  dp.on = true;
  dp.main = sub_pass{nullptr, nullptr, la, cnt, nullptr, 0, 0};
  dp.main.chain_of = reinterpret_cast<uint32_t *>(lg);
  dp.main.chain_rec = reinterpret_cast<uint32_t *>(lg + align_up(4 * cap, 256));
  dp.main.chain_end = dp.main.chain_rec + kChainCap;
  dp.main.nodes = reinterpret_cast<sub_node *>(dp.main.chain_end + kChainCap);
  dp.main.chain_cnt = cnt + 2;
  dp.main.node_cnt = cnt + 3;
  dp.main.chain_cap = kChainCap;
  dp.main.node_cap = kNodeCap;
  dp.main.heads = dp.main.nodes + kNodeCap;
  dp.A = sub_pass{la, cnt, lb, cnt + 1, sa, kDeepSlabA, 0};
  dp.B = sub_pass{lb, cnt + 1, nullptr, nullptr, sb, kDeepSlabB, 1};
  return XDRG_OK;
}

// The encode walk reuses the size pass's lists: it defers nothing.
deep_passes encode_passes(deep_passes dp) {
  if (!dp.on) return dp;
  dp.main.defer = nullptr;
  dp.main.defer_count = nullptr;
  dp.A.defer = nullptr;
  dp.A.defer_count = nullptr;
  return dp;
}

// The frame walks of a recursive plan: its generated module (codegen.cpp
// frame_walk_source) when the plan is specialized, else the interpreter.
const spec_module *frame_spec(const xdrg_plan &p) {
  if (!p.deep || !p.opts.specialize) return nullptr;
  const spec_module *m = spec_get(p);
  return m && m->f_sub_size ? m : nullptr;
}

// Launch kernel k, or the module function mf with the same parameters.
template <class... P, class TUP, size_t... I>
hipError_t module_launch(void *mf, uint32_t grid, uint32_t block, size_t lds, hipStream_t s, TUP &t,
                         std::index_sequence<I...>) {
  void *args[] = {static_cast<void *>(&std::get<I>(t))...};
  return hipModuleLaunchKernel(static_cast<hipFunction_t>(mf), grid, 1, 1, block, 1, 1, static_cast<uint32_t>(lds),
                               s, args, nullptr);
}
template <class... P, class... A>
hipError_t frame_launch(void (*k)(P...), void *mf, uint32_t grid, uint32_t block, size_t lds, hipStream_t s,
                        A... a) {
  if (!mf) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(block), lds, s, static_cast<P>(a)...);
    return hipGetLastError();
  }
  std::tuple<P...> t(static_cast<P>(a)...);  // the kernel's own parameter types
  return module_launch<P...>(mf, grid, block, lds, s, t, std::index_sequence_for<P...>{});
}

// The frame-walk size pass (k_sub_size) with its deep passes.
template <bool DEPTH>
hipError_t launch_sub_size(const xdrg_plan &p, const dev_tables &T, const uint8_t *nat, uint64_t n,
                           const uint8_t *heap, uint64_t heap_len, uint32_t *sizes, unsigned long long *bsum,
                           uint32_t mark, unsigned long long *err, uint32_t *depths, const deep_passes &dp,
                           hipStream_t s) {
  const size_t lds = p.ops.size() * sizeof(xdrg_op);
  const uint32_t nops = uint32_t(p.ops.size());
  const spec_module *FM = frame_spec(p);
  void *mf = FM ? (DEPTH ? FM->f_sub_depth : FM->f_sub_size) : nullptr;
  auto go = [&](uint32_t grid, uint32_t block, const sub_pass &P) {
    return frame_launch(k_sub_size<DEPTH>, mf, grid, block, lds, s, nat, n, p.stride, heap, heap_len,
                        T.d_ops, nops, T.d_table, sizes, bsum, mark, err, depths, P);
  };
  hipError_t e = go(static_cast<uint32_t>((n + 255) / 256), 256, dp.main);
  if (e == hipSuccess && dp.on && !DEPTH && dp.main.heads) {  // the chains the main pass handed over
    void *cf = FM ? FM->f_sub_chain_size : nullptr;
    e = frame_launch(k_sub_chain_size, cf, kChainGrid, 256, lds, s, nat, n, p.stride, heap, heap_len, T.d_ops, nops,
                     T.d_table, sizes, bsum, mark, err, depths, dp.main);
  }
  if (e == hipSuccess && dp.on) {
    e = go(kDeepLanesA / 256, 256, dp.A);
    if (e == hipSuccess) e = go(1, kDeepLanesB, dp.B);
  }
  return e;
}

hipError_t launch_size_pass(const xdrg_plan &p, const dev_tables &T, const uint8_t *nat, uint64_t n,
                            const uint8_t *heap, uint64_t heap_len, uint32_t *sizes,
                            unsigned long long *bsum, uint32_t mark, unsigned long long *err,
                            hipStream_t s, const deep_passes &dp = deep_passes{}) {
  if (p.has_sub)  // containers of variable-size elements: the frame walk
    return launch_sub_size<false>(p, T, nat, n, heap, heap_len, sizes, bsum, mark, err, nullptr, dp, s);
  if (p.linear && p.opts.size_linear != 0) {
    lin_args L;
    L.base = p.lin_base;
    L.n = p.lin_n;
    for (int k = 0; k < 8; ++k) L.off[k] = p.lin_off[k];
    k_size_linear<<<(n + 255) / 256, 256, 0, s>>>(nat, n, p.stride, L, sizes, bsum, mark, err);
    return hipGetLastError();
  }
  const uint64_t nb = (n + 63) / 64;
  const size_t tile = 64ull * p.stride;
  if (tile <= kVarLdsBudget)
    k_var_size<true><<<nb, 64, tile, s>>>(nat, n, p.stride, T.d_ops, uint32_t(p.ops.size()),
                                          T.d_table, sizes, bsum, mark, err);
  else
    k_var_size<false><<<nb, 64, 0, s>>>(nat, n, p.stride, T.d_ops, uint32_t(p.ops.size()),
                                        T.d_table, sizes, bsum, mark, err);
  return hipGetLastError();
}

unsigned long long *err_ptr(xdrg_status *st) {
  return reinterpret_cast<unsigned long long *>(&st->first_error);
}
}  // namespace

namespace {
__global__ __launch_bounds__(256) void k_fill32(uint32_t *__restrict__ p, uint32_t v, uint64_t words) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < words; i += stride) p[i] = v;
}
// 16-byte chunks when both ends allow it, else words, then the tail bytes
__global__ __launch_bounds__(256) void k_copy_bytes(uint8_t *__restrict__ d, const uint8_t *__restrict__ s,
                                                    uint64_t n) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint64_t done = 0;
  if (!((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s)) & 15u)) {
    const uint64_t c = n / 16;
    for (uint64_t i = t; i < c; i += stride)
      reinterpret_cast<u32x4 *>(d)[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(s) + i);
    done = c * 16;
  } else if (!((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s)) & 3u)) {
    const uint64_t c = n / 4;
    for (uint64_t i = t; i < c; i += stride)
      reinterpret_cast<uint32_t *>(d)[i] = reinterpret_cast<const uint32_t *>(s)[i];
    done = c * 4;
  }
  for (uint64_t i = done + t; i < n; i += stride) d[i] = s[i];
}
uint32_t copy_grid(uint64_t units) {  // a multiple of the 8 XCDs, at most 2,048 workgroups
  const uint64_t g = (units + 255) / 256;
  return static_cast<uint32_t>(std::max<uint64_t>(8, std::min<uint64_t>(2048, (g + 7) & ~7ull)));
}
}  // namespace

namespace xdrg {
int fill32(void *p, uint32_t value, uint64_t words, void *stream) {
  if (!words) return hipSuccess;
  k_fill32<<<copy_grid(words), 256, 0, static_cast<hipStream_t>(stream)>>>(static_cast<uint32_t *>(p), value, words);
  return hipGetLastError();
}
int copy_bytes(void *dst, const void *src, uint64_t n, void *stream) {
  if (!n) return hipSuccess;
  k_copy_bytes<<<copy_grid(n / 16 + 1), 256, 0, static_cast<hipStream_t>(stream)>>>(
      static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n);
  return hipGetLastError();
}
int launch_block_scan(const unsigned long long *in, unsigned long long *out, uint32_t nb,
                      xdrg_status *status, uint64_t *offsets, uint64_t n, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nb <= kScanMulti && in != out)
    k_scan_blocks<true><<<(nb + kScanNT - 1) / kScanNT, 1024, 0, s>>>(in, out, nb, status,
                                                                          offsets, n);
  else
    k_scan_blocks<false><<<1, 1024, 0, s>>>(in, out, nb, status, offsets, n);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}
int record_hip_error(int e, const char *what) { return hip_fail(static_cast<hipError_t>(e), what); }
}  // namespace xdrg

namespace {

// Var-plan encode of n records: size pass, block scan, then the record
// kernel.  mark = 4 puts each record in a message (its record mark first,
// xdrg_encode_msgs); mark = 0 is xdrg_encode of a var plan.  phase: both
// halves (kEncBoth), the size pass and scan alone into the workspace
// (kEncSizes, xdrg_encode_sizes: the total lands in status->total_bytes),
// or the record kernel over a workspace kEncSizes filled (kEncSized).
enum : int { kEncBoth = 0, kEncSizes = 1, kEncSized = 2 };
int var_encode(const xdrg_plan &P, const dev_tables &T, const void *d_native, uint64_t n,
               const uint8_t *d_heap, uint64_t heap_len, void *d_xdr, uint64_t cap,
               uint64_t *d_offsets, uint32_t stack_limit, void *d_ws, size_t ws_bytes,
               xdrg_status *d_status, uint32_t mark, hipStream_t s, int phase = kEncBoth) {
  const xdrg_plan *p = &P;
  const plan_opts &O = P.opts;
  unsigned long long *err = err_ptr(d_status);
  if (phase != kEncSizes && !d_offsets) return XDRG_EINVAL;
  if (d_heap && !aligned(d_heap, 4)) return XDRG_EALIGN;
  if (!aligned(d_native, 8) || (phase != kEncSizes && (!aligned(d_xdr, 4) || !aligned(d_offsets, 8))))
    return XDRG_EALIGN;
  if (n == 0) {
    if (d_offsets) HIPCHK(static_cast<hipError_t>(xdrg::fill32(d_offsets, 0u, 2, s)));
    return XDRG_OK;
  }
  size_t so, bo, bbo;
  const size_t need = var_ws_layout(n, &so, &bo, &bbo);
  if (!d_ws || ws_bytes < need + deep_area_bytes(*p, n)) return XDRG_ESPACE;
  uint32_t *sizes = reinterpret_cast<uint32_t *>(static_cast<char *>(d_ws) + so);
  unsigned long long *bsum = reinterpret_cast<unsigned long long *>(static_cast<char *>(d_ws) + bo);
  unsigned long long *bbase = reinterpret_cast<unsigned long long *>(static_cast<char *>(d_ws) + bbo);
  const uint64_t max_rec = p->max_record_bytes + mark;
  const uint32_t KI = p->max_var_slots <= 1 ? 1u : p->max_var_slots <= 2 ? 2u : 4u;
  // LDS window of the wave's output stretch (var_kernels.h): the stretch
  // leaves in rounds of C bytes, each round walking the records that reach
  // into it.  tools/tune/enc_stamps.py (MI355X, 1M records, plan-specialized
  // kernels): a cheap walk wants occupancy -- recvar (6 ops) 4 KiB 0.128 ms,
  // 8 KiB 0.139; a walk that loads container elements from the heap must not
  // repeat -- vecrec 8 KiB 0.159, 4 KiB 0.198; rpc (30 ops) 8 KiB 0.214,
  // 4 KiB 0.216.  Never more than the longest stretch needs.
  auto window = [&](void) -> uint32_t {
    const uint32_t want = O.image_bytes > 0 ? std::max(static_cast<uint32_t>(O.image_bytes) & ~15u, 256u)
                          : !p->has_vector && p->ops.size() <= 16 ? (4u << 10)
                                                                  : (8u << 10);
    return static_cast<uint32_t>(std::min<uint64_t>(want, (64ull * std::max<uint64_t>(max_rec, 16) + 31u) & ~15ull));
  };
  const uint32_t Ci = window();
  const enc_lds LI = enc_layout(p->stride, KI, Ci);
  const bool ok_I = p->max_var_slots <= 4 && 64ull * max_rec < (1ull << 31) && LI.total <= kVarLdsBudget &&
                    aligned(d_native, 16);
  int kern = O.enc_kernel;
  if (kern == 3 && !ok_I) kern = 0;
  if (kern == 0) kern = ok_I ? 3 : 1;
  const uint64_t nb = (n + 63) / 64;  // 64-record blocks for the size pass, scan and kernel 3
  if (nb > 0xffffffffull) return XDRG_EUNSUPPORTED;
  const size_t lds_ops = p->ops.size() * sizeof(xdrg_op);
  const uint8_t *nat8 = static_cast<const uint8_t *>(d_native);
  uint8_t *xdr8 = static_cast<uint8_t *>(d_xdr);
  const uint32_t nops = uint32_t(p->ops.size());
  // plan-specialized kernels (spec.cpp): straight-line size and encode walks
  const spec_module *SM = O.specialize && O.enc_kernel == 0 && !p->deep ? spec_get(*p) : nullptr;
  uint32_t Cs = 0, lds_s = 0;
  if (SM) {
    // a word-list walk (var_kernels.h WL) does not repeat per window, so
    // small windows cost no walks: rpc 4 KiB 0.169 ms vs 8 KiB 0.181,
    // recvar 4 KiB (profiles/r02s/ab_enc_wordlist_u*.log)
    Cs = p->spec.info.word_list && O.image_bytes <= 0
             ? static_cast<uint32_t>(std::min<uint64_t>(4u << 10, (64ull * std::max<uint64_t>(max_rec, 16) + 31u) & ~15ull))
             : window();
    // register walks without a word list load the record straight into
    // registers: no native tile (var_encode_body RREG)
    const bool rreg = p->spec.info.dec_regs && !p->spec.info.word_list;
    lds_s = enc_layout(rreg ? 0u : p->stride, p->spec.info.slots, Cs).total;
    // (a wave whose stretch could pass 2 GiB writes its records directly,
    // var_encode_body's direct mode)
    if (lds_s > kVarLdsBudget || !aligned(d_native, 16)) SM = nullptr;
  }
  // Word-list plans walked first (var_kernels.h var_encode_body, PRE): the
  // record kernel's walk runs once, before the windows, from registers and
  // without the checks (the plan's depth must fit the stack budget; a wave
  // stays under 2^31 bytes; a capacity re-walk lists its words in the
  // image), and it reads no sizes -- fewer registers than the per-window
  // walk (rpc 105 VGPRs vs 169): rpc size pass + scan + record kernel 0.155
  // ms vs 0.203, recvar 0.102 vs 0.103 (profiles/r04v).  XDRG_OPT_ENC_STREAM
  // 1 drops the size pass and scan as well, each wave's base from a
  // decoupled look-back over the totals of the waves before it: slower here
  // (rpc 0.262, recvar 0.187 ms): the polls cross the XCDs' L2s
  // (profiles/r04t).  The look-back over totals a size pass published first
  // (no wait on any wave's walk, no scan launch) is as slow: the record
  // kernel 189 vs 91 us for recvar, 218 vs 117 for rpc (profiles/r05p) --
  // the polls themselves, a kilobyte-window of uncached descriptor loads
  // per wave, cost more than the scan they replace.
  const bool pre = SM && SM->f_enc_pre && O.enc_stream != 0 && p->max_depth <= stack_limit &&
                   64ull * max_rec < (1ull << 31) && 256u * p->spec.info.list_words <= Cs;
  // its LDS: the word list in place of the native tile (var_encode_body PRE)
  const uint32_t lds_pre = pre ? enc_layout(4u * p->spec.info.list_words, p->spec.info.slots, Cs).total : 0u;
  if (pre && O.enc_stream == 1 && phase == kEncBoth) {
    uint64_t *total = &d_status->total_bytes;
    unsigned long long *desc = bsum;  // the nb wave totals (look-back descriptors)
    const unsigned long long *bb = bbase;
    uint32_t nb32 = static_cast<uint32_t>(nb), sl = stack_limit, cc = Cs, mk = mark;
    void *args[] = {&nat8, &n, const_cast<uint32_t *>(&p->stride), &d_heap, &heap_len, &xdr8, &cap,
                    &d_offsets, &bb, &desc, &nb32, &total, &sl, &cc, &mk, &err};
    HIPCHK(static_cast<hipError_t>(xdrg::fill32(desc, 0u, align_up(nb * 8, 16) / 4, s)));
    HIPCHK(hipModuleLaunchKernel(static_cast<hipFunction_t>(SM->f_enc_lb), nb32, 1, 1, 64, 1, 1, lds_pre, s, args,
                                 nullptr));
    return XDRG_OK;
  }
  deep_passes dp;  // element subroutines nested past XDRG_SUB_FRAMES
  if (p->has_sub)  // (the sized half walks the lists its size pass left in the workspace)
    if (int rc = deep_setup(*p, n, static_cast<char *>(d_ws) + need, ws_bytes - need, s, dp, phase != kEncSized))
      return rc;
  if (phase == kEncSized) {  // sizes and block bases from xdrg_encode_sizes
    HIPCHK(static_cast<hipError_t>(xdrg::copy_bytes(d_offsets + n, &d_status->total_bytes, 8, s)));
  } else {
    if (SM && (!p->linear || p->opts.size_linear != 1)) {  // (recvar: 12.2 vs k_size_linear's 13.2 us)
      const size_t tile = 64ull * p->stride;
      uint32_t n_mark = mark;
      void *args[] = {&nat8, &n, const_cast<uint32_t *>(&p->stride), &d_heap, &heap_len, &sizes, &bsum, &n_mark,
                      &err};
      HIPCHK(hipModuleLaunchKernel(static_cast<hipFunction_t>(SM->f_size), static_cast<uint32_t>(nb), 1, 1,
                                   64, 1, 1, static_cast<uint32_t>(tile), s, args, nullptr));
    } else {
      HIPCHK(launch_size_pass(*p, T, nat8, n, d_heap, heap_len, sizes, bsum, mark, err, s, dp));
    }
    if (int rc = xdrg::launch_block_scan(bsum, bbase, uint32_t(nb), d_status, d_offsets, n, s)) return rc;
    if (phase == kEncSizes) return XDRG_OK;
  }
  if (p->has_sub && !SM) {
    deep_passes ep = encode_passes(dp);
    const spec_module *FM = frame_spec(*p);
    void *mf = FM ? FM->f_sub_enc : nullptr;
    // the main pass's 64-byte line buffer per lane (sub_kernels.h
    // line_writer) when it fits beside the ops (plans up to ~1,500 ops);
    // past that the walk stores straight to the stream
    if (lds_ops > kVarLdsBudget) return XDRG_EUNSUPPORTED;
    ep.main.lines = lds_ops + 64u * 256u <= kVarLdsBudget ? 1u : 0u;
    auto go = [&](uint32_t grid, uint32_t block, const sub_pass &P) {  // + each lane's line buffer
      return frame_launch(k_sub_encode, mf, grid, block, lds_ops + (P.lines ? 64u * block : 0u), s, nat8, n,
                          p->stride, d_heap,
                          heap_len, xdr8, cap, d_offsets, sizes, bbase, T.d_ops, nops, T.d_table, stack_limit, mark,
                          err, P);
    };
    HIPCHK(go(static_cast<uint32_t>((n + 255) / 256), 256, ep.main));
    if (ep.on) {
      HIPCHK(go(kDeepLanesA / 256, 256, ep.A));
      HIPCHK(go(1, kDeepLanesB, ep.B));
      // the node pass: the logged chains' nodes (sub_kernels.h "Chains")
      void *cf = FM ? FM->f_sub_chain : nullptr;
      HIPCHK(frame_launch(k_sub_chain, cf, kChainGrid, 256, lds_ops, s, nat8, n, p->stride, d_heap, heap_len, xdr8,
                          cap, d_offsets, sizes, bbase, T.d_ops, nops, T.d_table, stack_limit, mark, err, ep.main));
    }
    return XDRG_OK;
  }
  if (pre) {  // the walk-first record kernel over the scan's wave bases
    const unsigned long long *bb = bbase;
    unsigned long long *nodesc = nullptr;
    uint64_t *nototal = nullptr;
    uint32_t nb32 = static_cast<uint32_t>(nb), sl = stack_limit, cc = Cs, mk = mark;
    void *args[] = {&nat8, &n, const_cast<uint32_t *>(&p->stride), &d_heap, &heap_len, &xdr8, &cap,
                    &d_offsets, &bb, &nodesc, &nb32, &nototal, &sl, &cc, &mk, &err};
    HIPCHK(hipModuleLaunchKernel(static_cast<hipFunction_t>(SM->f_enc_pre), nb32, 1, 1, 64, 1, 1, lds_pre, s, args,
                                 nullptr));
    return XDRG_OK;
  }
  if (SM) {
    const unsigned long long *bb = bbase;
    uint32_t sl = stack_limit, cc = Cs, mk = mark;
    void *args[] = {&nat8, &n, const_cast<uint32_t *>(&p->stride), &d_heap, &heap_len, &xdr8, &cap,
                    &d_offsets, &sizes, &bb, &sl, &cc, &mk, &err};
    HIPCHK(hipModuleLaunchKernel(static_cast<hipFunction_t>(SM->f_enc), static_cast<uint32_t>(nb), 1, 1, 64, 1,
                                 1, lds_s, s, args, nullptr));
    return XDRG_OK;
  }
  if (kern == 3) {
#define LAUNCH_ENC_IU(K, UU)                                                                   \
  k_var_encode_i<K, UU><<<nb, 64, LI.total, s>>>(nat8, n, p->stride, d_heap, heap_len, xdr8,  \
                                                 cap, d_offsets, sizes, bbase, T.d_ops, nops,   \
                                                 T.d_table, stack_limit, Ci, mark, err)
#define LAUNCH_ENC_I(K)                                     \
  do {                                                      \
    if (O.enc_unroll == 16) LAUNCH_ENC_IU(K, 16);           \
    else if (O.enc_unroll == 4) LAUNCH_ENC_IU(K, 4);        \
    else LAUNCH_ENC_IU(K, 8);                               \
  } while (0)
    if (KI == 1) LAUNCH_ENC_I(1);
    else if (KI == 2) LAUNCH_ENC_I(2);
    else LAUNCH_ENC_I(4);
#undef LAUNCH_ENC_I
#undef LAUNCH_ENC_IU
    HIPCHK(hipGetLastError());
    return XDRG_OK;
  }
  const uint64_t nb256 = (n + 255) / 256;
  k_var_encode<<<nb256, 256, lds_ops, s>>>(nat8, n, p->stride, d_heap, heap_len, xdr8, cap, d_offsets,
                                           sizes, bbase, T.d_ops, nops, T.d_table, stack_limit, mark,
                                           err);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

// Index pass levels and workspace: per level L (n[L] nodes) a table of
// n[L] * K words (below the top) and n[L] entry words.
struct ix_layout {
  uint64_t nseg = 0;
  size_t list = 0, lcount = 0;  // valid-node lists (kIxSW words per segment) and their lengths
  uint32_t K = 0, F = 0;
  bool lds = false;
  int top = 0;
  uint64_t n[24] = {};
  size_t tab[24] = {}, pf[24] = {}, ent[24] = {};
  uint64_t rxs_nseg = 0;  // fast path (record index): segments, their records,
  size_t rxs_seg = 0, rxs_cnt = 0, rxs_base = 0, rxs_tot = 0, rxs_flag = 0;  // counts, bases, total, flag
                          // (its node lists: in the list area)
  size_t total = 0;
};
constexpr size_t kIxLdsBytes = 64u << 10;
constexpr size_t kIxNextBytes = 256;  // ix_windows' continuation block

ix_layout ix_plan(uint64_t len, uint32_t maxlen) {
  ix_layout L;
  L.nseg = (len / 4) / kIxSW + 1;  // covers the end-of-stream word
  L.K = maxlen / 4 + 1;
  L.F = L.K <= 128 ? 64 : 16;
  L.lds = static_cast<size_t>(L.F) * L.K * 8 <= kIxLdsBytes;
  L.n[0] = L.nseg;
  while (L.n[L.top] > 1) {
    L.n[L.top + 1] = (L.n[L.top] + L.F - 1) / L.F;
    ++L.top;
  }
  size_t off = 0;
  L.list = off;
  off += align_up(L.nseg * kIxSW * 4, 256);
  L.lcount = off;
  off += align_up(L.nseg * 4, 256);
  for (int l = 0; l <= L.top; ++l) {
    if (l < L.top) {
      L.tab[l] = off;
      off += align_up(L.n[l] * L.K * 8, 256);
      L.pf[l] = off;  // prefix compositions (k_ix_up) of the same shape
      off += align_up(L.n[l] * L.K * 8, 256);
    }
    L.ent[l] = off;
    off += align_up(L.n[l] * 8, 256);
  }
  L.rxs_nseg = (len + kRxsSeg - 1) / kRxsSeg;  // its u16 node lists fit the list area
  L.rxs_seg = off;
  off += align_up(L.rxs_nseg * kRxsSegWords * 8, 256);
  L.rxs_cnt = off;
  off += align_up(L.rxs_nseg * 8, 256);
  L.rxs_base = off;
  off += align_up(L.rxs_nseg * 8, 256);
  L.rxs_tot = off;
  off += 256;
  L.rxs_flag = off;  // the workspace's last 256 bytes (include/xdrgpu.h)
  off += 256;
  L.total = off;
  return L;
}

// Heap bytes a decode needs; plans without payload or element fields need
// none when decoding messages (the decoded records hold no heap refs).
bool plan_has_payload(const xdrg_plan &p) { return p.max_var_slots > 0 || p.has_vector; }

// Var-plan decode of n records indexed by d_offsets (mark = 4: each record
// is a message whose mark is checked, xdrg_decode_msgs).
int var_decode(const xdrg_plan &P, const dev_tables &T, const void *d_xdr, uint64_t len,
               const uint64_t *d_offsets, uint64_t n, void *d_native, uint8_t *d_heap_out,
               uint64_t heap_cap, uint32_t stack_limit, xdrg_status *d_status, uint32_t mark,
               void *d_ws, size_t ws_bytes, hipStream_t s) {
  const xdrg_plan *p = &P;
  const plan_opts &O = P.opts;
  unsigned long long *err = err_ptr(d_status);
  if (n == 0) {
    if (len) return launch_report(err, 0, kOpRecordLevel, XDRG_ERR_TRAILING, s);
    return XDRG_OK;
  }
  bool no_heap = false;
  if (mark && !d_heap_out && !plan_has_payload(*p)) {  // nothing points into a heap
    d_heap_out = static_cast<uint8_t *>(const_cast<void *>(d_xdr));
    no_heap = true;
  }
  if (!no_heap && (heap_cap < decode_heap_bytes(*p, len) || (len && !d_heap_out)))
    return XDRG_ESPACE;
  const uint64_t ebase = p->has_vector ? align_up(len, 16) : 0;  // decoded element arrays
  if (!aligned(d_xdr, 4) || !aligned(d_native, 8) || (d_heap_out && !aligned(d_heap_out, 4)))
    return XDRG_EALIGN;
  const uint8_t *xdr8 = static_cast<const uint8_t *>(d_xdr);
  uint8_t *nat8 = static_cast<uint8_t *>(d_native);
  const uint32_t nops = uint32_t(p->ops.size());
  const bool copy = d_heap_out != d_xdr;  // heap_out == d_xdr: zero-copy (refs into the stream)
  // LDS window: tools/tune/enc_stamps.py (OPT=window_bytes, MI355X, 1M
  // records).  Plans with a short walk are bound by the global reads of the
  // records past the window: a 16 KiB window (recvar's whole ~12 KiB
  // stretch) cut recvar's decode 0.120 -> 0.089 ms, vecrec's 0.222 ->
  // 0.216.  A long walk (rpc, 30 ops) wants the occupancy instead: 4 KiB
  // (0.142 ms) beats 8 KiB (0.154) and 16 KiB (0.164).
  const uint32_t win = O.window_bytes >= 0 ? static_cast<uint32_t>(O.window_bytes) & ~15u
                       : p->ops.size() <= 16 ? (16u << 10)
                       : 64ull * (len / n) <= (8u << 10) ? (8u << 10) : (4u << 10);
  const uint32_t Cw = static_cast<uint32_t>(std::min<uint64_t>(
      win, (64ull * std::max<uint64_t>(p->max_record_bytes + mark, 16) + 15u) & ~15ull));
  // Stage of a group's element arrays (packed plans, var_kernels.h
  // var_decode_body).  tools/tune/dec_ab.py (MI355X, vecrec 1M records,
  // profiles/r03q): no stage 0.137 ms and 348 MiB written per launch; an
  // 8 KiB stage (every group's arrays fit) with an 8 KiB window 0.138 ms and
  // 276 MiB -- the algorithmic bytes (0.128 ms once the stage leaves with
  // non-temporal stores, profiles/r03s); a 12 KiB stage or a 16 KiB window
  // cost occupancy (0.148-0.182 ms), a window below the 64 records' ~6.6
  // KiB stretch sends the walk to global memory (0.188 ms at 6 KiB).
  const uint32_t S = !p->packed ? 0u
                     : O.stage_bytes >= 0 ? static_cast<uint32_t>(O.stage_bytes) & ~15u : (8u << 10);
  const uint32_t lw = dec_w_lds(p->stride, Cw, false, S);
  const bool ok_W = lw <= kVarLdsBudget && aligned(d_native, 16);
  int kern = O.dec_kernel;
  if (kern == 2 && !ok_W) kern = 0;
  if (kern == 0) kern = ok_W ? 2 : 1;
  const spec_module *SM = O.specialize && O.dec_kernel == 0 && kern == 2 && !p->deep ? spec_get(*p) : nullptr;
  if (p->has_sub && !SM) {  // containers of variable-size elements: the frame walk
    deep_passes dp;  // element subroutines nested past XDRG_SUB_FRAMES
    if (int rc = deep_setup(*p, n, d_ws, ws_bytes, s, dp)) return rc;
    if (copy && len) HIPCHK(static_cast<hipError_t>(xdrg::copy_bytes(d_heap_out, d_xdr, len, s)));
    const size_t lds = p->ops.size() * sizeof(xdrg_op);
    const spec_module *FM = frame_spec(*p);
    void *mf = FM ? FM->f_sub_dec : nullptr;
    auto go = [&](uint32_t grid, uint32_t block, const sub_pass &P) {
      return frame_launch(k_sub_decode, mf, grid, block, lds, s, xdr8, len, d_offsets, n, nat8, p->stride, T.d_ops,
                          nops, T.d_table, stack_limit, d_heap_out, ebase, p->heap_factor, mark, err, P);
    };
    sub_pass mp = dp.main;
    mp.packed = p->packed ? 1u : 0u;  // non-recursive plans: packed element areas (never deferred)
    // the waves' stream windows (sub_kernels.h win_rd) and the wave pass
    // take kWaveWaves * kWaveBlk bytes of LDS beside the ops: a plan whose
    // ops leave no room for them (about 1,000 ops) walks its long records
    // in the main pass, as without the wave pass
    const size_t lds_win = align_up(lds, 16) + size_t(kWaveWaves) * kWaveBlk;
    const bool wave = dp.on && lds_win <= kVarLdsBudget;
    if (wave) {  // long records to the wave pass
      mp.wave_list = dp.main.chain_of;
      mp.wave_count = dp.main.defer_count + 4;
    }
    mp.win = wave ? 1u : 0u;
    HIPCHK(frame_launch(k_sub_decode, mf, static_cast<uint32_t>((n + 255) / 256), 256, wave ? lds_win : lds, s,
                        xdr8, len, d_offsets, n, nat8, p->stride, T.d_ops, nops, T.d_table, stack_limit,
                        d_heap_out, ebase, p->heap_factor, mark, err, mp));
    if (wave) {
      sub_pass W{};
      W.list = mp.wave_list;
      W.count = mp.wave_count;
      W.defer = dp.main.defer;  // what its frames cannot finish: deep pass A
      W.defer_count = dp.main.defer_count;
      W.wave = 1;
      // linked lists' node candidates (sub_kernels.h list_decode), when the
      // ops leave room for them
      const size_t lds_list = lds_win + size_t(kWaveWaves) * (kWaveBlk / 2);
      W.win = lds_list <= kVarLdsBudget ? 1u : 0u;
      HIPCHK(frame_launch(k_sub_decode, mf, kWaveGrid, 64 * kWaveWaves, W.win ? lds_list : lds_win, s, xdr8, len,
                          d_offsets, n, nat8,
                          p->stride, T.d_ops, nops, T.d_table, stack_limit, d_heap_out, ebase, p->heap_factor, mark,
                          err, W));
    }
    if (dp.on) {
      HIPCHK(go(kDeepLanesA / 256, 256, dp.A));
      HIPCHK(go(1, kDeepLanesB, dp.B));
    }
    return XDRG_OK;
  }
  if (SM) {  // plan-specialized decode walk (spec.cpp)
    const uint64_t nb = (n + 63) / 64;
    uint32_t st = p->stride, sl = stack_limit, cw = Cw, F = p->heap_factor, mk = mark, lws = lw;
    if (p->spec.info.dec_regs) {
      // no native tile in LDS: the window gets its room.  tools/tune/
      // enc_stamps.py (OPT=window_bytes, MI355X, 1M records,
      // profiles/r02s/ab_dec_window*.log): rpc 4 KiB 0.159 ms, 8 KiB 0.146,
      // 16 KiB 0.126, 20 KiB 0.128, 32 KiB 0.177; recvar and vecrec are
      // flat from 16 KiB (0.089, 0.226) and slower below
      const uint32_t want = O.window_bytes >= 0 ? static_cast<uint32_t>(O.window_bytes) & ~15u
                            : S ? (8u << 10) : (16u << 10);  // (packed: the stage above)
      cw = static_cast<uint32_t>(std::min<uint64_t>(
          want, (64ull * std::max<uint64_t>(p->max_record_bytes + mark, 16) + 15u) & ~15ull));
      lws = dec_w_lds(p->stride, cw, true, S);
    } else {
      lws = dec_w_lds(p->stride, cw, false, S);
    }
    uint64_t eb = ebase;
    uint32_t sb = S;
    void *args[] = {&xdr8, &len, &d_offsets, &n, &nat8, &st, &d_heap_out, &sl, &cw, &eb, &F, &mk, &sb, &err};
    HIPCHK(hipModuleLaunchKernel(static_cast<hipFunction_t>(copy ? SM->f_dec_copy : SM->f_dec),
                                 static_cast<uint32_t>(nb), 1, 1, 64, 1, 1, lws, s, args, nullptr));
    return XDRG_OK;
  }
  if (kern == 2) {
    const uint64_t nb = (n + 63) / 64;
#define LAUNCH_DEC_W(CP, RA)                                                                      \
  k_var_decode_w<CP, RA><<<nb, 64, lw, s>>>(xdr8, len, d_offsets, n, nat8, p->stride, d_heap_out, \
                                            T.d_ops, nops, T.d_table, stack_limit, Cw, ebase,     \
                                            p->heap_factor, mark, p->packed, S, err)
    if (copy) {
      if (O.dec_readahead) LAUNCH_DEC_W(true, true); else LAUNCH_DEC_W(true, false);
    } else {
      if (O.dec_readahead) LAUNCH_DEC_W(false, true); else LAUNCH_DEC_W(false, false);
    }
#undef LAUNCH_DEC_W
  } else {
    if (copy && len) HIPCHK(static_cast<hipError_t>(xdrg::copy_bytes(d_heap_out, d_xdr, len, s)));
    const uint64_t nb = (n + 255) / 256;
    k_var_decode<<<nb, 256, p->ops.size() * sizeof(xdrg_op), s>>>(
        xdr8, len, d_offsets, n, nat8, p->stride, T.d_ops, nops, T.d_table, stack_limit,
        d_heap_out, ebase, p->heap_factor, mark, p->packed, err);
  }
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

}  // namespace

namespace {
constexpr int kIxNotHeld = 1;  // run_index(fast_only): the speculative walk did not hold
// C: the window of a longer stream this index covers (ix_cont); the
// offsets, count and errors are the whole stream's.  fast_only: the
// speculative walk alone (XDRG_OK when it holds the index, kIxNotHeld when
// it did not run or a check failed; nothing reported either way).
template <bool REC>
int run_index(const xdrg_plan *p, const dev_tables *T, const void *d_stream, uint64_t len,
              uint32_t max_msg_len, uint64_t max_msgs, uint64_t *d_offsets, uint64_t *d_count,
              void *d_ws, size_t ws_bytes, xdrg_status *d_status, hipStream_t s,
              const ix_cont &C = ix_cont{}, bool fast_only = false, bool whole = false) {
  const ix_layout L = ix_plan(len, max_msg_len);
  if (!d_ws || ws_bytes < L.total) return XDRG_ESPACE;
  if (L.nseg > 0xffffffffull) return XDRG_EUNSUPPORTED;
  rx_plan rp{REC ? T->d_ops : nullptr, REC ? T->d_table : nullptr, REC ? uint32_t(p->ops.size()) : 0u,
             RX_BAD, 0};
  if (REC) {  // the first checked op: fixed-size ops before it, no branch
    uint32_t d = 0;
    for (uint32_t pc = 0; pc < p->ops.size(); ++pc) {
      const xdrg_op &o = p->ops[pc];
      if (o.kind == XDRG_OP_END || o.kind == XDRG_OP_JUMP) break;
      if (o.kind == XDRG_OP_U64) { d += 8; continue; }
      if (o.kind == XDRG_OP_OPAQUE) { d += (o.arg0 + 3u) & ~3u; continue; }
      if (o.kind == XDRG_OP_U32 || o.kind == XDRG_OP_BOOL ||
          (o.kind == XDRG_OP_ENUM && !(o.flags & XDRG_F_VALIDATE))) { d += 4; continue; }
      rp.fpc = pc;
      rp.fd = d;
      break;
    }
  }
  const size_t ops_lds = REC ? p->ops.size() * sizeof(xdrg_op) : 0;
  if (ops_lds > (38u << 10)) return XDRG_EUNSUPPORTED;  // + 25 KiB static: the 64 KiB workgroup LDS
  unsigned long long *err = err_ptr(d_status);
  char *ws = static_cast<char *>(d_ws);
  auto tab = [&](int l) { return reinterpret_cast<uint64_t *>(ws + L.tab[l]); };
  auto ent = [&](int l) { return reinterpret_cast<uint64_t *>(ws + L.ent[l]); };
  const uint8_t *s8 = static_cast<const uint8_t *>(d_stream);
  uint32_t *vlist = reinterpret_cast<uint32_t *>(ws + L.list);
  uint32_t *vcount = reinterpret_cast<uint32_t *>(ws + L.lcount);
  // the tables are needed above one segment; the valid-node lists always
  // record starts: the plan's generated parse when its kernels are built
  // (codegen.cpp plan_rx), else the interpreted rx_len
  // (recursive plans: a linked list's generated parse, codegen.cpp tail_list)
  const spec_module *SM = REC && p->opts.specialize ? spec_get(*p) : nullptr;
  if (SM && !SM->f_rxs_walk) SM = nullptr;
  // whole: the walk over records of any length (rx_windows): its parse has
  // no maxlen, and a record past the staged stretch is parsed by the wave
  if (whole && !(SM && SM->f_rxs_walk_whole && SM->f_rxs_fix)) whole = false;
  // Record index: the speculative chain walk first (index_kernels.h rxs_*);
  // the list ranking below runs only when its checks fail.  Short streams
  // (a few segments) go to the list ranking alone.
  const uint32_t *skip = nullptr;
  // (with the plan's generated parse: the interpreted one makes the walk
  // slower than the list ranking -- rpc 0.65 vs 0.45 ms, vecrec 0.79 vs
  // 0.25, its op loop and frame stack on every candidate -- so a plan
  // without specialized kernels takes the list ranking)
  // Message streams walk their marks (mark_rx) always.
  const bool walk_ok = REC ? SM && SM->f_rxs_walk && p->opts.index_fast : true;
  int gate = REC ? p->opts.index_fast : 1;
  const bool walk_only = gate == 3;  // (a tuning aid: the walk's records stay in the workspace)
  if (walk_only) gate = 1;
  if (gate == 1) {  // a stream being captured into a graph cannot be waited on: stay asynchronous
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) gate = 2;
  }
  if (fast_only) gate = 1;  // ix_windows: the walk's verdict, nothing else
  const bool walk_runs = walk_ok && !C.next && len >= 4ull * kRxsSeg && max_msgs > 0;
  // the count's fill for the list ranking (a window's caller sets it once):
  // after the walk's verdict when the host waits for it (no launch when the
  // walk holds: its emit writes the count), else first
  const bool fill_late = walk_runs && gate == 1 && !fast_only && !walk_only;
  if (!C.next && !fill_late) HIPCHK(static_cast<hipError_t>(xdrg::fill32(d_count, 0xffffffffu, 2, s)));
  if (fast_only && !walk_runs) return kIxNotHeld;
  if (REC && !C.next && !walk_runs)  // the flag says which path ran (include/xdrgpu.h)
    HIPCHK(static_cast<hipError_t>(xdrg::fill32(ws + L.rxs_flag, 0u, 1, s)));
  if (walk_runs) {
    uint64_t *seg = reinterpret_cast<uint64_t *>(ws + L.rxs_seg);
    auto *cnt = reinterpret_cast<unsigned long long *>(ws + L.rxs_cnt);
    auto *base = reinterpret_cast<unsigned long long *>(ws + L.rxs_base);
    auto *tot = reinterpret_cast<xdrg_status *>(ws + L.rxs_tot);
    uint32_t *flag = reinterpret_cast<uint32_t *>(ws + L.rxs_flag);
    uint16_t *nodes = reinterpret_cast<uint16_t *>(vlist);  // the list ranking's lists, unused when it skips
    const uint32_t ns = static_cast<uint32_t>(L.rxs_nseg);
    if (REC) {
      uint32_t ml = whole ? 0xffffffffu : max_msg_len, hf = rp.fpc != RX_BAD, fd = rp.fd;
      void *args[] = {&s8, &len, &ml, &seg, &nodes, &flag, &hf, &fd};
      HIPCHK(hipModuleLaunchKernel(static_cast<hipFunction_t>(whole ? SM->f_rxs_walk_whole : SM->f_rxs_walk), ns, 1,
                                   1, 64, 1, 1, 0, s, args, nullptr));
    } else {
      k_rxs_walk_msgs<<<ns, 64, 0, s>>>(s8, len, max_msg_len, seg, nodes, flag);
      HIPCHK(hipGetLastError());
    }
    if (whole) {
      // the failed segments' list in the scan's output area (written after
      // the fix), its count a u64 at flag + 2 (zeroed by the walk)
      uint64_t *list = reinterpret_cast<uint64_t *>(base);
      auto *nl = reinterpret_cast<unsigned long long *>(flag + 2);
      k_rxs_check<true><<<(ns + 255) / 256, 256, 0, s>>>(seg, nodes, L.rxs_nseg, len, cnt, flag, list, nl);
      HIPCHK(hipGetLastError());
      uint32_t ml = 0xffffffffu;
      uint64_t nsg = L.rxs_nseg;
      void *jargs[] = {&s8, &len, &ml, &seg, &nsg, &nodes, &list, &nl, &flag, &cnt};
      HIPCHK(hipModuleLaunchKernel(static_cast<hipFunction_t>(SM->f_rxs_fix), 1, 1, 1, 64, 1, 1, 0, s, jargs,
                                   nullptr));
    } else {
      k_rxs_check<false><<<(ns + 255) / 256, 256, 0, s>>>(seg, nodes, L.rxs_nseg, len, cnt, flag, nullptr, nullptr);
      HIPCHK(hipGetLastError());
    }
    if (int rc = launch_block_scan(cnt, base, ns, tot, nullptr, 0, s)) return rc;
    // the verdict also into this thread's mapped host word (gate 1): the
    // host waits for the stream alone, no copy after the kernels
    uint32_t *hw = gate == 1 ? host_verdict_word() : nullptr;
    uint32_t *hwd = nullptr;
    if (hw && hipHostGetDevicePointer(reinterpret_cast<void **>(&hwd), hw, 0) != hipSuccess) hwd = nullptr;
    if (hwd) *reinterpret_cast<volatile uint32_t *>(hw) = 0xffffffffu;
    k_rxs_emit<REC><<<(ns + kRxsEmitWaves - 1) / kRxsEmitWaves, 64 * kRxsEmitWaves, 0, s>>>(
        seg, nodes, base, tot, len, max_msgs, d_offsets, d_count, flag, L.rxs_nseg, hwd, cnt);
    HIPCHK(hipGetLastError());
    if (gate == 1) {
      // wait for the flag: the list ranking is launched only when a check
      // failed (its ~11 launches would otherwise cost ~45 us of skipping)
      uint32_t h = 0;
      if (hwd) {
        HIPCHK(hipStreamSynchronize(s));
        h = *reinterpret_cast<volatile uint32_t *>(hw);
      } else {
        HIPCHK(hipMemcpyAsync(&h, flag, sizeof h, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
      }
      if (h == 1u) return XDRG_OK;
      if (fast_only) return kIxNotHeld;
      if (walk_only) return XDRG_OK;
      if (fill_late) HIPCHK(static_cast<hipError_t>(xdrg::fill32(d_count, 0xffffffffu, 2, s)));
    } else {
      skip = flag;  // asynchronous: the list ranking's kernels skip themselves
    }
  }
  if (SM && SM->f_ix_seg) {
    uint64_t *t0 = L.top > 0 ? tab(0) : nullptr;
    uint32_t ml = max_msg_len, K = L.K, hf = rp.fpc != RX_BAD, fd = rp.fd;
    void *args[] = {&s8, &len, &ml, &K, &t0, &vlist, &vcount, &hf, &fd, &skip};
    HIPCHK(hipModuleLaunchKernel(static_cast<hipFunction_t>(SM->f_ix_seg), static_cast<uint32_t>(L.nseg), 1, 1, 256,
                                 1, 1, 0, s, args, nullptr));
  } else {
    k_ix_seg<REC><<<L.nseg, 256, ops_lds, s>>>(s8, len, max_msg_len, L.K, L.top > 0 ? tab(0) : nullptr,
                                               vlist, vcount, rp, skip);
    HIPCHK(hipGetLastError());
  }
  const size_t stg = L.lds ? static_cast<size_t>(L.F) * L.K * 8 : 0;
  auto pfx = [&](int l) { return reinterpret_cast<uint64_t *>(ws + L.pf[l]); };
  for (int l = 0; l < L.top; ++l) {  // the top level: prefixes only
    uint64_t *o = l + 1 < L.top ? tab(l + 1) : nullptr;
    if (L.lds)
      k_ix_up<true><<<L.n[l + 1], 256, stg, s>>>(tab(l), L.n[l], L.K, L.F, o, pfx(l), skip);
    else
      k_ix_up<false><<<L.n[l + 1], 256, 0, s>>>(tab(l), L.n[l], L.K, L.F, o, pfx(l), skip);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(static_cast<hipError_t>(xdrg::fill32(ent(L.top), 0u, 2, s)));  // the chain starts at word 0 with 0 messages
  for (int l = L.top - 1; l >= 0; --l) {
    k_ix_down<<<L.n[l + 1], 64, 0, s>>>(pfx(l), L.n[l], L.K, L.F, ent(l + 1), ent(l), skip);
    HIPCHK(hipGetLastError());
  }
  k_ix_emit<REC><<<L.nseg, 256, 0, s>>>(s8, len, max_msg_len, ent(0), vlist, vcount, d_offsets + C.m0,
                                        max_msgs - C.m0, reinterpret_cast<unsigned long long *>(d_count), err,
                                        rp, C, skip);
  HIPCHK(hipGetLastError());
  if (REC && !C.next) {  // (rx_windows fills once, after its last round)
    k_rx_fill<<<static_cast<uint32_t>(std::min<uint64_t>((max_msgs + 256) / 256, 4096)), 256, 0, s>>>(
        d_offsets, reinterpret_cast<const unsigned long long *>(d_count), max_msgs, len, skip);
    HIPCHK(hipGetLastError());
  }
  return XDRG_OK;
}

// Message index of a stream whose messages may be longer than one index
// window (max_msg_len > XDRG_INDEX_MAX_MSG; msg_sock's default is 1 MiB,
// msgsock.h:29, and read_message has no limit, srpc.cc:29-55).  Rounds,
// each picking up where the chain left the last one:
//   k_ix_long  walks the long messages from there, mark after mark;
//   a window   the list-ranking index (run_index, messages up to
//              XDRG_INDEX_MAX_MSG) over the stream from the first short
//              message on, until its chain reaches a long message or the
//              window's end (ix_final leaves the continuation).
// The first window is the whole stream, so a stream without long messages
// takes one round.  A window that its chain left early is followed by one
// twice as long as the stretch the chain covered (at least kIxMinWindow):
// the index reads each byte about twice at most, plus two host waits per
// round (the continuation is read back).
constexpr uint64_t kIxMinWindow = 1ull << 20;
int ix_windows(const uint8_t *s8, uint64_t len, uint32_t max_msg_len, uint64_t max_msgs, uint64_t *d_offsets,
               uint64_t *d_count, void *d_ws, size_t ws_bytes, xdrg_status *d_status, hipStream_t s) {
  const size_t need = xdrg_index_workspace_size(len, max_msg_len);
  if (!d_ws || ws_bytes < need) return XDRG_ESPACE;
  {  // the rounds wait on the stream: a stream being captured cannot be waited on
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return XDRG_EUNSUPPORTED;
  }
  // A stream whose messages all fit one index window (the usual case under
  // msg_sock's 1 MiB default) is indexed by the speculative mark walk of
  // run_index alone; any long message, or a check that fails, leaves it to
  // the rounds below, which rewrite the count and every offset.
  {
    const int rc = run_index<false>(nullptr, nullptr, s8, len, XDRG_INDEX_MAX_MSG, max_msgs, d_offsets, d_count,
                                    d_ws, ws_bytes, d_status, s, ix_cont{}, true);
    if (rc != kIxNotHeld) return rc;
  }
  auto *next = reinterpret_cast<unsigned long long *>(static_cast<char *>(d_ws) + need - kIxNextBytes);
  unsigned long long *err = err_ptr(d_status);
  unsigned long long *count = reinterpret_cast<unsigned long long *>(d_count);
  HIPCHK(static_cast<hipError_t>(xdrg::fill32(d_count, 0xffffffffu, 2, s)));
  HIPCHK(static_cast<hipError_t>(xdrg::fill32(next, 0u, 6, s)));  // the chain starts at word 0, message 0
  unsigned long long h[3] = {0, 0, 0};
  uint64_t window = len;
  for (;;) {
    k_ix_long<<<1, 64, 0, s>>>(s8, len, max_msg_len, max_msgs, d_offsets, count, err, next, 4096u);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h, next, 24, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h[0] == ~0ull) return XDRG_OK;
    if (!h[2]) continue;  // the hop budget ran out among long messages
    const uint64_t start = 4 * h[0], m0 = h[1];
    const uint64_t wl = std::min<uint64_t>(window, len - start);
    HIPCHK(static_cast<hipError_t>(xdrg::fill32(next, 0xffffffffu, 2, s)));
    const ix_cont C{m0, start, s8, len, max_msg_len, next};
    if (int rc = run_index<false>(nullptr, nullptr, s8 + start, wl, XDRG_INDEX_MAX_MSG, max_msgs, d_offsets,
                                  d_count, d_ws, ws_bytes, d_status, s, C))
      return rc;
    HIPCHK(hipMemcpyAsync(h, next, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h[0] == ~0ull) return XDRG_OK;
    const uint64_t covered = 4 * h[0] - start;
    window = covered < wl ? std::max<uint64_t>(2 * covered, kIxMinWindow) : 2 * wl;
  }
}

// Record index of a stream with records longer than one index window
// (max_rec_len > XDRG_INDEX_MAX_MSG) or nested deeper than its frames: the
// rounds of ix_windows over records.  k_rx_long walks such records from
// where the chain stopped; a list-ranking window (run_index over records
// up to XDRG_INDEX_MAX_MSG bytes) indexes the stream from the next record
// until its chain reaches one again or the window's end.  The speculative
// walk tries the whole stream first.
int rx_windows(const xdrg_plan *p, const dev_tables *T, const uint8_t *s8, uint64_t len, uint64_t n,
               uint64_t *d_offsets, uint64_t *d_count, void *d_ws, size_t ws_bytes, xdrg_status *d_status,
               hipStream_t s) {
  const size_t need = xdrg_index_workspace_size(len, XDRG_INDEX_MAX_MSG + 4u);
  if (!d_ws || ws_bytes < need) return XDRG_ESPACE;
  {  // the rounds wait on the stream: a stream being captured cannot be waited
     // on.  There the walk over the whole stream runs alone, asynchronously:
     // when its checks fail the list ranking over records up to the window
     // follows (its kernels skip themselves otherwise), which reports
     // XDRG_ERR_INDEX_LONG at a longer record
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
      const spec_module *SM = p->opts.specialize ? spec_get(*p) : nullptr;
      if (!(SM && SM->f_rxs_walk_whole && SM->f_rxs_fix && p->opts.index_fast))
        return XDRG_EUNSUPPORTED;
      return run_index<true>(p, T, s8, len, XDRG_INDEX_MAX_MSG, n, d_offsets, d_count, d_ws, ws_bytes, d_status, s,
                             ix_cont{}, false, true);
    }
  }
  {  // the speculative walk over the whole stream, records of any length (a
     // plan with the generated parse: the walk parses the long ones); else
     // over records up to the index window
    const int rc = run_index<true>(p, T, s8, len, XDRG_INDEX_MAX_MSG, n, d_offsets, d_count, d_ws, ws_bytes,
                                   d_status, s, ix_cont{}, true, true);
    if (rc != kIxNotHeld) return rc;
    if (p->opts.index_fast == 3) return XDRG_OK;  // the walk alone (XDRG_OPT_INDEX_FAST)
  }
  const ix_layout L0 = ix_plan(len, XDRG_INDEX_MAX_MSG);
  auto *next = reinterpret_cast<unsigned long long *>(static_cast<char *>(d_ws) + L0.total);
  auto *slab = reinterpret_cast<rx_frame *>(static_cast<char *>(d_ws) + L0.total + kIxNextBytes);
  unsigned long long *count = reinterpret_cast<unsigned long long *>(d_count);
  HIPCHK(static_cast<hipError_t>(xdrg::fill32(d_count, 0xffffffffu, 2, s)));
  HIPCHK(static_cast<hipError_t>(xdrg::fill32(next, 0u, 6, s)));  // the chain starts at word 0, record 0
  unsigned long long h[3] = {0, 0, 0};
  // the long-record walk's ops in LDS (up to 1,024 ops)
  const uint32_t nops = static_cast<uint32_t>(p->ops.size());
  const uint32_t ops_lds = nops <= 1024u ? nops * static_cast<uint32_t>(sizeof(xdrg_op)) : 0u;
  uint64_t window = len;
  for (;;) {
    k_rx_long<<<1, 64, ops_lds, s>>>(s8, len, XDRG_INDEX_MAX_MSG, n, T->d_ops, T->d_table, d_offsets, count, next,
                                     slab, 256u, nops, ops_lds ? 1u : 0u);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h, next, 24, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h[0] == ~0ull) break;
    if (!h[2]) continue;  // the hop budget ran out among long records
    const uint64_t start = 4 * h[0], m0 = h[1];
    const uint64_t wl = std::min<uint64_t>(window, len - start);
    HIPCHK(static_cast<hipError_t>(xdrg::fill32(next, 0xffffffffu, 2, s)));
    const ix_cont C{m0, start, s8, len, XDRG_INDEX_MAX_MSG, next};
    if (int rc = run_index<true>(p, T, s8 + start, wl, XDRG_INDEX_MAX_MSG, n, d_offsets, d_count, d_ws, ws_bytes,
                                 d_status, s, C))
      return rc;
    HIPCHK(hipMemcpyAsync(h, next, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h[0] == ~0ull) break;
    const uint64_t covered = 4 * h[0] - start;
    window = covered < wl ? std::max<uint64_t>(2 * covered, kIxMinWindow) : 2 * wl;
  }
  k_rx_fill<<<static_cast<uint32_t>(std::min<uint64_t>((n + 256) / 256, 4096)), 256, 0, s>>>(
      d_offsets, reinterpret_cast<const unsigned long long *>(d_count), n, len, nullptr);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}
}  // namespace

// ==================================================================== C ABI
extern "C" {

int xdrg_abi_version(void) { return XDRG_ABI_VERSION; }

const char *xdrg_last_hip_error(void) { return g_hip_err; }

int xdrg_plan_create(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t ntable,
                     uint32_t native_stride, xdrg_plan **out) {
  if (!ops || !out || nops == 0 || (ntable && !table)) return XDRG_EINVAL;
  *out = nullptr;
  // status keys carry 16 bits of op index, 0xffff meaning "record level"
  if (nops >= kOpRecordLevel) return XDRG_EUNSUPPORTED;
  xdrg_plan *p = new (std::nothrow) xdrg_plan();
  if (!p) return XDRG_ENOMEM;
  p->ops.assign(ops, ops + nops);
  if (ntable) p->table.assign(table, table + ntable);
  p->stride = native_stride;
  int rc = xdrg::compile_plan(*p);
  if (rc != XDRG_OK) { delete p; return rc; }
  if (p->stride % 4) { delete p; return XDRG_EUNSUPPORTED; }
  *out = p;
  return XDRG_OK;
}

int xdrg_plan_set_option(xdrg_plan *p, int option, int64_t value) {
  if (!p) return XDRG_EINVAL;
  plan_opts &O = p->opts;
  const int v = static_cast<int>(value);
  if (value != v) return XDRG_EINVAL;
  switch (option) {
  case XDRG_OPT_VAR_ENCODE_KERNEL:
    if (v != 0 && v != 1 && v != 3) return XDRG_EINVAL;
    O.enc_kernel = v; return XDRG_OK;
  case XDRG_OPT_VAR_DECODE_KERNEL:
    if (v < 0 || v > 2) return XDRG_EINVAL;
    O.dec_kernel = v; return XDRG_OK;
  case XDRG_OPT_FIXED_PATH:
    if (v != 0 && v != 2 && v != 3) return XDRG_EINVAL;
    O.fixed_path = v; return XDRG_OK;
  case XDRG_OPT_IMAGE_BYTES:
    if (v > (32 << 10)) return XDRG_EINVAL;
    O.image_bytes = v < 0 ? -1 : v; return XDRG_OK;
  case XDRG_OPT_WINDOW_BYTES:
    if (v > (32 << 10)) return XDRG_EINVAL;
    O.window_bytes = v < 0 ? -1 : v; return XDRG_OK;
  case XDRG_OPT_ENC_UNROLL:
    if (v != 4 && v != 8 && v != 16) return XDRG_EINVAL;
    O.enc_unroll = v; return XDRG_OK;
  case XDRG_OPT_DEC_READAHEAD: O.dec_readahead = v ? 1 : 0; return XDRG_OK;
  case XDRG_OPT_SIZE_LINEAR: O.size_linear = v < 0 ? -1 : v ? 1 : 0; return XDRG_OK;
  case XDRG_OPT_GRP_UNROLL:
    if (v != 0 && v != 1 && v != 2 && v != 4) return XDRG_EINVAL;
    O.grp_unroll = v; return XDRG_OK;
  case XDRG_OPT_GRP_BLOCKS:
    if (v < 0) return XDRG_EINVAL;
    O.grp_blocks = v; return XDRG_OK;
  case XDRG_OPT_GRP_NONTEMPORAL: O.grp_nontemporal = v ? 1 : 0; return XDRG_OK;
  case XDRG_OPT_SPECIALIZE: O.specialize = v ? 1 : 0; return XDRG_OK;
  case XDRG_OPT_INDEX_FAST:
    if (v < 0 || v > 3) return XDRG_EINVAL;
    O.index_fast = static_cast<int>(v); return XDRG_OK;
  case XDRG_OPT_STAGE_BYTES:
    if (v > (32 << 10)) return XDRG_EINVAL;
    O.stage_bytes = v < 0 ? -1 : v; return XDRG_OK;
  case XDRG_OPT_ENC_STREAM:
    if (v < -1 || v > 1) return XDRG_EINVAL;
    O.enc_stream = static_cast<int>(v); return XDRG_OK;
  case XDRG_OPT_FIXED_STREAM:
    if (v < -1 || v > 3) return XDRG_EINVAL;
    O.fixed_stream = v; return XDRG_OK;
  default: return XDRG_EINVAL;
  }
}

// The plan's tables on the current device: one allocation holding every
// table, made by the plan's first launch on that device.
static int plan_upload(const xdrg_plan *cp, const dev_tables **out) {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) return XDRG_EUNSUPPORTED;
  xdrg_plan *p = const_cast<xdrg_plan *>(cp);
  *out = &p->dev[dev];
  if (p->uploaded[dev].load(std::memory_order_acquire)) return XDRG_OK;
  std::lock_guard<std::mutex> g(p->upload_mu);
  if (p->uploaded[dev].load(std::memory_order_relaxed)) return XDRG_OK;
  struct part { const void *src; size_t bytes; size_t off; };
  part parts[12] = {
      {p->ops.data(), p->ops.size() * sizeof(xdrg_op), 0},
      {p->table.data(), p->table.size() * 4, 0},
      {p->enc.idx.data(), p->enc.idx.size() * sizeof(term_idx), 0},
      {p->enc.terms.data(), p->enc.terms.size() * sizeof(term), 0},
      {p->dec.idx.data(), p->dec.idx.size() * sizeof(term_idx), 0},
      {p->dec.terms.data(), p->dec.terms.size() * sizeof(term), 0},
      {p->enc.reg.data(), p->enc.reg.size() * sizeof(reg_word), 0},
      {p->dec.reg.data(), p->dec.reg.size() * sizeof(reg_word), 0},
      {p->checks.data(), p->checks.size() * sizeof(check), 0},
      {p->enc.grp.data(), p->enc.grp.size() * sizeof(grp_term), 0},
      {p->dec.grp.data(), p->dec.grp.size() * sizeof(grp_term), 0},
      {nullptr, 16, 0}};
  size_t total = 0;
  for (part &q : parts) { q.off = total; total += align_up(q.bytes, 256); }
  void *mem = nullptr;
  hipError_t e = hipMalloc(&mem, total);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(plan)");
  char *base = static_cast<char *>(mem);
  for (part &q : parts)
    if (q.src && q.bytes) {
      e = hipMemcpy(base + q.off, q.src, q.bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) { (void)hipFree(mem); return hip_fail(e, "hipMemcpy(plan)"); }
    }
  dev_tables &T = p->dev[dev];
  T.d_mem = mem;
  T.d_ops = reinterpret_cast<const xdrg_op *>(base + parts[0].off);
  T.d_table = reinterpret_cast<const uint32_t *>(base + parts[1].off);
  T.d_enc_idx = reinterpret_cast<const term_idx *>(base + parts[2].off);
  T.d_enc_terms = reinterpret_cast<const term *>(base + parts[3].off);
  T.d_dec_idx = reinterpret_cast<const term_idx *>(base + parts[4].off);
  T.d_dec_terms = reinterpret_cast<const term *>(base + parts[5].off);
  T.d_enc_reg = reinterpret_cast<const reg_word *>(base + parts[6].off);
  T.d_dec_reg = reinterpret_cast<const reg_word *>(base + parts[7].off);
  T.d_checks = reinterpret_cast<const check *>(base + parts[8].off);
  T.d_enc_grp = reinterpret_cast<const grp_term *>(base + parts[9].off);
  T.d_dec_grp = reinterpret_cast<const grp_term *>(base + parts[10].off);
  p->uploaded[dev].store(true, std::memory_order_release);
  return XDRG_OK;
}

void xdrg_plan_destroy(xdrg_plan *p) {
  if (!p) return;
  xdrg::spec_release(p->spec);
  int cur = 0;
  const bool restore = hipGetDevice(&cur) == hipSuccess;
  for (int d = 0; d < kMaxDevices; ++d)
    if (p->dev[d].d_mem) {
      (void)hipSetDevice(d);
      (void)hipFree(p->dev[d].d_mem);
    }
  if (restore) (void)hipSetDevice(cur);
  delete p;
}

int xdrg_plan_get_info(const xdrg_plan *p, xdrg_plan_info *info) {
  if (!p || !info) return XDRG_EINVAL;
  info->path = p->path;
  info->native_stride = p->stride;
  info->fixed_size = p->fixed_size;
  info->max_depth = p->max_depth;
  info->nops = uint32_t(p->ops.size());
  info->has_checks = p->has_checks ? 1u : 0u;
  info->max_record_bytes = p->max_record_bytes;
  info->group_records = p->path == XDRG_PATH_FIXED_LDS && !p->has_checks ? p->enc.grp_G : 0u;
  int dev = 0;
  const bool failed_here = hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kSpecDevices &&
                           p->spec.failed[dev].load();
  info->specialized = p->spec.state.load() == 1 && !failed_here ? 1u : 0u;
  return XDRG_OK;
}

uint64_t xdrg_decode_heap_size(const xdrg_plan *p, uint64_t len) {
  return p ? decode_heap_bytes(*p, len) : 0;
}

size_t xdrg_workspace_size(const xdrg_plan *p, uint64_t n) {
  if (!p) return 0;  // var encode of any plan; encode_msgs of every plan
  size_t a, b;
  return var_ws_layout(n, &a, &b) + deep_area_bytes(*p, n);
}

size_t xdrg_deep_workspace_size(const xdrg_plan *p, uint64_t n) { return p ? deep_area_bytes(*p, n) : 0; }

int xdrg_status_init(xdrg_status *st, void *stream) {
  if (!st) return XDRG_EINVAL;
  HIPCHK(static_cast<hipError_t>(xdrg::fill32(st, 0xffffffffu, 2, stream)));
  HIPCHK(static_cast<hipError_t>(xdrg::fill32(reinterpret_cast<char *>(st) + 8, 0u, 2, stream)));
  return XDRG_OK;
}

int xdrg_status_read(const xdrg_status *st, void *stream, xdrg_error *out) {
  if (!st || !out) return XDRG_EINVAL;
  HIPCHK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  xdrg_status h;
  HIPCHK(hipMemcpy(&h, st, sizeof h, hipMemcpyDeviceToHost));
  memset(out, 0, sizeof *out);
  out->total_bytes = h.total_bytes;
  if (h.first_error == ~0ull) return XDRG_OK;
  out->code = int32_t(h.first_error & 0xff);
  out->op = uint32_t((h.first_error >> 8) & 0xffff);
  if (out->op == kOpRecordLevel) out->op = 0xffffffffu;
  out->record = h.first_error >> 24;
  out->exc = xdrg_error_exception(out->code);
  return XDRG_OK;
}

int xdrg_encode(const xdrg_plan *p, const void *d_native, uint64_t n, const uint8_t *d_heap,
                uint64_t heap_len, void *d_xdr, uint64_t cap, uint64_t *d_offsets,
                uint32_t stack_limit, void *d_ws, size_t ws_bytes, xdrg_status *d_status,
                void *stream) {
  if (!p || !d_status || (n && (!d_native || !d_xdr))) return XDRG_EINVAL;
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  unsigned long long *err = err_ptr(d_status);
  if (p->path != XDRG_PATH_VAR) {
    if (n == 0) return XDRG_OK;
    if (p->max_depth > stack_limit)  // every record fails at the same op
      return launch_report(err, 0, first_op_deeper(*p, stack_limit), XDRG_ERR_STACK_PUT, s);
    const uint64_t W = p->fixed_size;
    uint64_t nrec = n;
    if (cap < n * W) {
      nrec = cap / W;
      int rc = launch_report(err, nrec, first_op_past(*p, cap - nrec * W), XDRG_ERR_OVERFLOW_PUT, s);
      if (rc) return rc;
    }
    if (d_offsets) return XDRG_EINVAL;  // fixed plans: offsets are implied
    return run_fixed(*p, *T, false, d_native, d_xdr, nrec, err, s);
  }
  // ---- variable plans
  return var_encode(*p, *T, d_native, n, d_heap, heap_len, d_xdr, cap, d_offsets, stack_limit, d_ws,
                    ws_bytes, d_status, 0u, s);
}

int xdrg_decode(const xdrg_plan *p, const void *d_xdr, uint64_t len, const uint64_t *d_offsets,
                uint64_t n, void *d_native, uint8_t *d_heap_out, uint64_t heap_cap,
                uint32_t stack_limit, void *d_ws, size_t ws_bytes, xdrg_status *d_status,
                void *stream) {
  if (!p || !d_status || (n && (!d_native || (len && !d_xdr)))) return XDRG_EINVAL;
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  unsigned long long *err = err_ptr(d_status);
  if (p->path != XDRG_PATH_VAR) {
    if (len & 3u)  // xdr_generic_get ctor, marshal.h:155-160
      return launch_report(err, 0, kOpRecordLevel, XDRG_ERR_SIZE_NOT_MULT4, s);
    if (n == 0) {
      if (len) return launch_report(err, 0, kOpRecordLevel, XDRG_ERR_TRAILING, s);
      return XDRG_OK;
    }
    if (p->max_depth > stack_limit)
      return launch_report(err, 0, first_op_deeper(*p, stack_limit), XDRG_ERR_STACK_GET, s);
    const uint64_t W = p->fixed_size;
    uint64_t nrec = n;
    if (len < n * W) {
      nrec = len / W;
      int rc = launch_report(err, nrec, first_op_past(*p, len - nrec * W), XDRG_ERR_OVERFLOW_GET, s);
      if (rc) return rc;
    } else if (len > n * W) {
      int rc = launch_report(err, n, kOpRecordLevel, XDRG_ERR_TRAILING, s);
      if (rc) return rc;
    }
    return run_fixed(*p, *T, true, d_xdr, d_native, nrec, err, s);
  }
  if (!d_offsets) return XDRG_EUNSUPPORTED;  // var decode needs a record index
  return var_decode(*p, *T, d_xdr, len, d_offsets, n, d_native, d_heap_out, heap_cap, stack_limit,
                    d_status, 0u, d_ws, ws_bytes, s);
}

int xdrg_record_depths(const xdrg_plan *p, const void *d_native, uint64_t n, const void *d_heap,
                       uint64_t heap_len, uint32_t *d_depths, void *d_ws, size_t ws_bytes,
                       xdrg_status *d_status, void *stream) {
  if (!p || !d_status || (n && (!d_native || !d_depths))) return XDRG_EINVAL;
  if (n == 0) return XDRG_OK;
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p->has_sub) {
    deep_passes dp;  // element subroutines nested past XDRG_SUB_FRAMES
    if (int rc = deep_setup(*p, n, d_ws, ws_bytes, s, dp)) return rc;
    HIPCHK(launch_sub_size<true>(*p, *T, static_cast<const uint8_t *>(d_native), n,
                                 static_cast<const uint8_t *>(d_heap), heap_len, nullptr, nullptr, 0u,
                                 err_ptr(d_status), d_depths, dp, s));
    return XDRG_OK;
  }
  if (p->path != XDRG_PATH_VAR || p->linear) {  // every record walks every op
    HIPCHK(static_cast<hipError_t>(xdrg::fill32(d_depths, p->max_depth, n, s)));
    return XDRG_OK;
  }
  const uint64_t nb = (n + 63) / 64;
  const size_t tile = 64ull * p->stride;
  const uint8_t *nat = static_cast<const uint8_t *>(d_native);
  unsigned long long *err = err_ptr(d_status);
  if (tile <= kVarLdsBudget)
    k_var_size<true, true><<<nb, 64, tile, s>>>(nat, n, p->stride, T->d_ops, uint32_t(p->ops.size()),
                                                T->d_table, nullptr, nullptr, 0u, err, d_depths);
  else
    k_var_size<false, true><<<nb, 64, 0, s>>>(nat, n, p->stride, T->d_ops, uint32_t(p->ops.size()),
                                              T->d_table, nullptr, nullptr, 0u, err, d_depths);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

int xdrg_serial_sizes(const xdrg_plan *p, const void *d_native, uint64_t n, const void *d_heap,
                      uint64_t heap_len, uint32_t *d_sizes, uint32_t stack_limit, void *d_ws,
                      size_t ws_bytes, xdrg_status *d_status, void *stream) {
  (void)stack_limit;
  if (!p || !d_status || (n && (!d_native || !d_sizes))) return XDRG_EINVAL;
  if (n == 0) return XDRG_OK;
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p->path != XDRG_PATH_VAR) {
    // fixed_size for every record (xdr_struct_base_fs, types.h:691-700)
    HIPCHK(static_cast<hipError_t>(xdrg::fill32(d_sizes, p->fixed_size, n, s)));
    return XDRG_OK;
  }
  deep_passes dp;  // element subroutines nested past XDRG_SUB_FRAMES
  if (p->has_sub)
    if (int rc = deep_setup(*p, n, d_ws, ws_bytes, s, dp)) return rc;
  HIPCHK(launch_size_pass(*p, *T, static_cast<const uint8_t *>(d_native), n,
                          static_cast<const uint8_t *>(d_heap), heap_len, d_sizes, nullptr, 0u,
                          err_ptr(d_status), s, dp));
  return XDRG_OK;
}

int xdrg_encode_msgs(const xdrg_plan *p, const void *d_native, uint64_t n, const uint8_t *d_heap,
                     uint64_t heap_len, void *d_out, uint64_t cap, uint64_t *d_offsets,
                     uint32_t stack_limit, void *d_ws, size_t ws_bytes, xdrg_status *d_status,
                     void *stream) {
  if (!p || !d_status || (n && (!d_native || !d_out))) return XDRG_EINVAL;
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  return var_encode(*p, *T, d_native, n, d_heap, heap_len, d_out, cap, d_offsets, stack_limit, d_ws,
                    ws_bytes, d_status, 4u, static_cast<hipStream_t>(stream));
}

int xdrg_encode_sizes(const xdrg_plan *p, const void *d_native, uint64_t n, const uint8_t *d_heap,
                      uint64_t heap_len, uint32_t stack_limit, int msgs, void *d_ws, size_t ws_bytes,
                      xdrg_status *d_status, void *stream) {
  if (!p || !d_status || (n && !d_native)) return XDRG_EINVAL;
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p->path != XDRG_PATH_VAR && !msgs) {  // n * fixed_size (xdr_struct_base_fs, types.h:691-700)
    k_set_total<<<1, 1, 0, s>>>(d_status, n * uint64_t(p->fixed_size));
    HIPCHK(hipGetLastError());
    return XDRG_OK;
  }
  return var_encode(*p, *T, d_native, n, d_heap, heap_len, nullptr, 0, nullptr, stack_limit, d_ws, ws_bytes,
                    d_status, msgs ? 4u : 0u, s, kEncSizes);
}

int xdrg_encode_sized(const xdrg_plan *p, const void *d_native, uint64_t n, const uint8_t *d_heap,
                      uint64_t heap_len, void *d_out, uint64_t cap, uint64_t *d_offsets, uint32_t stack_limit,
                      int msgs, void *d_ws, size_t ws_bytes, xdrg_status *d_status, void *stream) {
  if (!p || !d_status || (n && (!d_native || !d_out))) return XDRG_EINVAL;
  if (p->path != XDRG_PATH_VAR && !msgs)
    return xdrg_encode(p, d_native, n, d_heap, heap_len, d_out, cap, d_offsets, stack_limit, d_ws, ws_bytes,
                       d_status, stream);
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  return var_encode(*p, *T, d_native, n, d_heap, heap_len, d_out, cap, d_offsets, stack_limit, d_ws, ws_bytes,
                    d_status, msgs ? 4u : 0u, static_cast<hipStream_t>(stream), kEncSized);
}

size_t xdrg_index_workspace_size(uint64_t len, uint32_t max_msg_len) {
  if (max_msg_len > XDRG_MAX_MSG) return 0;
  if (max_msg_len <= XDRG_INDEX_MAX_MSG) return ix_plan(len, max_msg_len).total;
  // + the windows' continuation and the long-record walk's frames (rx_windows)
  return ix_plan(len, XDRG_INDEX_MAX_MSG).total + kIxNextBytes + sizeof(rx_frame) * size_t(XDRG_MAX_FRAMES);
}

int xdrg_index_msgs(const void *d_stream, uint64_t len, uint32_t max_msg_len, uint64_t max_msgs,
                    uint64_t *d_offsets, uint64_t *d_count, void *d_ws, size_t ws_bytes,
                    xdrg_status *d_status, void *stream) {
  if (!d_offsets || !d_count || !d_status || (len && !d_stream)) return XDRG_EINVAL;
  if (max_msg_len > XDRG_MAX_MSG) return XDRG_EINVAL;
  if ((d_stream && !aligned(d_stream, 4)) || !aligned(d_offsets, 8) || !aligned(d_count, 8))
    return XDRG_EALIGN;
  if (max_msgs >= (1ull << 40)) return XDRG_EUNSUPPORTED;  // entry words hold 40-bit counts
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (max_msg_len <= XDRG_INDEX_MAX_MSG)
    return run_index<false>(nullptr, nullptr, d_stream, len, max_msg_len, max_msgs, d_offsets, d_count,
                            d_ws, ws_bytes, d_status, s);
  return ix_windows(static_cast<const uint8_t *>(d_stream), len, max_msg_len, max_msgs, d_offsets, d_count,
                    d_ws, ws_bytes, d_status, s);
}

int xdrg_index_records(const xdrg_plan *p, const void *d_xdr, uint64_t len, uint64_t n,
                       uint32_t max_rec_len, uint64_t *d_offsets, uint64_t *d_count, void *d_ws,
                       size_t ws_bytes, xdrg_status *d_status, void *stream) {
  if (!p || !d_offsets || !d_count || !d_status || (len && !d_xdr)) return XDRG_EINVAL;
  if (max_rec_len > XDRG_MAX_MSG) return XDRG_EINVAL;
  if ((d_xdr && !aligned(d_xdr, 4)) || !aligned(d_offsets, 8) || !aligned(d_count, 8)) return XDRG_EALIGN;
  if (n >= (1ull << 40)) return XDRG_EUNSUPPORTED;
  if (p->min_record_bytes < 4) return XDRG_EUNSUPPORTED;  // the chain must advance
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  if (max_rec_len > XDRG_INDEX_MAX_MSG)
    return rx_windows(p, T, static_cast<const uint8_t *>(d_xdr), len, n, d_offsets, d_count, d_ws, ws_bytes,
                      d_status, static_cast<hipStream_t>(stream));
  return run_index<true>(p, T, d_xdr, len, max_rec_len, n, d_offsets, d_count, d_ws, ws_bytes, d_status,
                         static_cast<hipStream_t>(stream));
}



int xdrg_decode_msgs(const xdrg_plan *p, const void *d_stream, uint64_t len,
                     const uint64_t *d_offsets, uint64_t n, void *d_native, uint8_t *d_heap_out,
                     uint64_t heap_cap, uint32_t stack_limit, void *d_ws, size_t ws_bytes,
                     xdrg_status *d_status, void *stream) {
  if (!p || !d_status || !d_offsets || (n && (!d_native || (len && !d_stream)))) return XDRG_EINVAL;
  const dev_tables *T = nullptr;
  if (int rc = plan_upload(p, &T)) return rc;
  return var_decode(*p, *T, d_stream, len, d_offsets, n, d_native, d_heap_out, heap_cap, stack_limit,
                    d_status, 4u, d_ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int xdrg_swap32(const uint32_t *in, uint32_t *out, uint64_t n, void *stream) {
  if (n && (!in || !out)) return XDRG_EINVAL;
  if (!n) return XDRG_OK;
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
  k_swap32<<<blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(in, out, n);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

int xdrg_swap64(const uint64_t *in, uint64_t *out, uint64_t n, void *stream) {
  if (n && (!in || !out)) return XDRG_EINVAL;
  if (!n) return XDRG_OK;
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
  k_swap64<<<blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(in, out, n);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

const char *xdrg_error_message(int code) {
  switch (code) {
  case XDRG_ERR_NONE: return "";
  case XDRG_ERR_OVERFLOW_GET: return "insufficient buffer space in xdr_generic_get";
  case XDRG_ERR_OVERFLOW_PUT: return "insufficient buffer space in xdr_generic_put";
  case XDRG_ERR_XVECTOR_BOUND: return "xvector overflow";
  case XDRG_ERR_XSTRING_BOUND: return "xstring overflow";
  case XDRG_ERR_NONZERO_PAD: return "Non-zero padding bytes encountered";
  case XDRG_ERR_BAD_DISCRIMINANT: return "bad value of discriminant";
  case XDRG_ERR_INVALID_ENUM: return "Invalid enum value";
  case XDRG_ERR_STACK_PUT: return "stack overflow in xdr_generic_put";
  case XDRG_ERR_STACK_GET: return "stack overflow in xdr_generic_get";
  case XDRG_ERR_SIZE_NOT_MULT4: return "xdr_generic_get: message size not multiple of 4";
  case XDRG_ERR_TRAILING: return "unmarshaling did not consume whole message";
  case XDRG_ERR_POINTER_BOUND: return "xdr::pointer size must be 0 or 1";
  case XDRG_ERR_MSG_EOF: return "read_message: premature EOF";
  case XDRG_ERR_MSG_SIZE4: return "read_message: received size not multiple of 4";
  case XDRG_ERR_MSG_FRAGMENT: return "read_message: message fragments unimplemented";
  case XDRG_ERR_MSG_TOO_LONG: return "msg_sock: rejecting message (too long)";
  case XDRG_ERR_MSG_MISMATCH: return "record mark does not match the record index";
  case XDRG_ERR_MSG_COUNT: return "more messages than the record index holds";
  case XDRG_ERR_INDEX_LONG: return "record longer than the device record index window";
  case XDRG_ERR_LOOKBACK: return "one-pass encode: look-back timed out (internal error)";
  default: return "unknown xdrgpu error";
  }
}

int xdrg_error_exception(int code) {
  switch (code) {
  case XDRG_ERR_OVERFLOW_GET: case XDRG_ERR_OVERFLOW_PUT: case XDRG_ERR_XVECTOR_BOUND:
  case XDRG_ERR_XSTRING_BOUND: case XDRG_ERR_POINTER_BOUND: return XDRG_EXC_OVERFLOW;
  case XDRG_ERR_NONZERO_PAD: return XDRG_EXC_SHOULD_BE_ZERO;
  case XDRG_ERR_BAD_DISCRIMINANT: return XDRG_EXC_BAD_DISCRIMINANT;
  case XDRG_ERR_INVALID_ENUM: return XDRG_EXC_INVARIANT_FAILED;
  case XDRG_ERR_STACK_PUT: case XDRG_ERR_STACK_GET: return XDRG_EXC_STACK_OVERFLOW;
  case XDRG_ERR_SIZE_NOT_MULT4: case XDRG_ERR_TRAILING: return XDRG_EXC_BAD_MESSAGE_SIZE;
  // read_message throws xdr_bad_message_size (srpc.cc:36-52); msg_sock's
  // rejections (no exception there, msgsock.cc:86-117) map to the same class
  case XDRG_ERR_MSG_EOF: case XDRG_ERR_MSG_SIZE4: case XDRG_ERR_MSG_FRAGMENT:
  case XDRG_ERR_MSG_TOO_LONG: case XDRG_ERR_MSG_MISMATCH: case XDRG_ERR_MSG_COUNT:
    return XDRG_EXC_BAD_MESSAGE_SIZE;
  default: return XDRG_EXC_NONE;
  }
}

}  // extern "C"
