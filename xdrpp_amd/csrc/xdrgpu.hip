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

#include "plan.h"

using namespace xdrg;

namespace {

thread_local char g_hip_err[256] = "";

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
using namespace xdrg::dev;

namespace {

// ------------------------------------------------------------ var: helpers
__device__ __forceinline__ uint32_t ld32(const uint8_t *p) {
  return *reinterpret_cast<const uint32_t *>(p);
}
__device__ __forceinline__ void st32(uint8_t *p, uint32_t v) {
  *reinterpret_cast<uint32_t *>(p) = v;
}

// Little-endian word made of the 4 bytes at [p + off, p + off + 4) of a
// 4-byte-aligned buffer of `len` bytes; bytes at or past `len` read as 0.
__device__ __forceinline__ uint32_t partial_word(const uint8_t *p, uint64_t len, uint64_t a) {
  uint32_t v = 0;
  for (uint32_t k = 0; k < 4; ++k)
    if (a + k < len) v |= static_cast<uint32_t>(p[a + k]) << (8 * k);
  return v;
}
__device__ __forceinline__ uint32_t unaligned_word(const uint8_t *p, uint64_t len, uint64_t off) {
  const uint64_t a = off & ~3ull;
  const uint32_t sh = static_cast<uint32_t>(off & 3u);
  const uint32_t lo = (a + 4 <= len) ? ld32(p + a) : partial_word(p, len, a);
  if (sh == 0) return lo;
  const uint32_t hi = (a + 8 <= len) ? ld32(p + a + 4) : partial_word(p, len, a + 4);
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
__device__ __forceinline__ uint32_t keep_mask(uint32_t nbytes) {  // nbytes in 1..4
  return nbytes >= 4 ? 0xffffffffu : ((1u << (8u * nbytes)) - 1u);
}

__device__ __forceinline__ int union_target(const xdrg_op &op, const uint32_t *__restrict__ table,
                                            uint32_t d) {
  for (uint32_t i = 0; i < op.arg3; ++i)
    if (table[op.arg2 + 2 * i] == d) return static_cast<int>(table[op.arg2 + 2 * i + 1]);
  return (op.flags & XDRG_F_DEFAULT) ? static_cast<int>(op.arg4) : -1;
}

__device__ __forceinline__ void load_ops(xdrg_op *sops, const xdrg_op *__restrict__ ops,
                                         uint32_t nops) {
  const uint32_t *s = reinterpret_cast<const uint32_t *>(ops);
  uint32_t *d = reinterpret_cast<uint32_t *>(sops);
  for (uint32_t i = threadIdx.x; i < nops * 8u; i += blockDim.x) d[i] = s[i];
  __syncthreads();
}

constexpr uint32_t kSizeErr = 0x80000000u;

// -------------------------------------------------------- var: size pass
// xdr_traits<T>::serial_size per record and bad discriminants
// (gen_hh.cc:639-648).  The stack budget is a put-side check
// (marshal.h:129-136) and is applied by k_var_encode.
__global__ __launch_bounds__(256) void k_var_size(const uint8_t *__restrict__ native, uint64_t n,
                                                  uint32_t stride, const xdrg_op *__restrict__ ops,
                                                  uint32_t nops, const uint32_t *__restrict__ table,
                                                  uint32_t *__restrict__ sizes,
                                                  unsigned long long *__restrict__ block_sums,
                                                  unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  __shared__ unsigned long long wsum[4];
  load_ops(sops, ops, nops);
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint32_t size = 0;
  if (r < n) {
    const uint8_t *nat = native + r * stride;
    uint64_t s = 0;
    uint32_t pc = 0, bad_op = 0xffffffffu;
    for (;;) {
      const xdrg_op &op = sops[pc];
      if (op.kind == XDRG_OP_END) break;
      if (op.kind == XDRG_OP_JUMP) { pc = op.arg0; continue; }
      switch (op.kind) {
      case XDRG_OP_U64: s += 8; ++pc; break;
      case XDRG_OP_OPAQUE: s += (op.arg0 + 3u) & ~3u; ++pc; break;
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
        s += 4u + ((static_cast<uint64_t>(ld32(nat + op.noff + 8)) + 3u) & ~3ull);
        ++pc;
        break;
      case XDRG_OP_UNION: {
        const int t = union_target(op, table, ld32(nat + op.noff));
        s += 4;
        if (t < 0) { bad_op = pc; goto done; }
        pc = static_cast<uint32_t>(t);
        break;
      }
      default: s += 4; ++pc; break;
      }
    }
  done:
    if (bad_op != 0xffffffffu) {
      report(err, r, bad_op, XDRG_ERR_BAD_DISCRIMINANT);
      size = kSizeErr;
    } else if (s >= kSizeErr) {
      report(err, r, 0, XDRG_ERR_OVERFLOW_PUT);
      size = kSizeErr;
    } else {
      size = static_cast<uint32_t>(s);
    }
    sizes[r] = size;
  }
  // block sum of the valid sizes
  unsigned long long v = (size & kSizeErr) ? 0ull : size;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (uint32_t w = 0; w < (blockDim.x + 63) / 64; ++w) t += wsum[w];
    block_sums[blockIdx.x] = t;
  }
}

// Exclusive scan of nb block sums in place; writes the total.
__global__ __launch_bounds__(1024) void k_scan_blocks(unsigned long long *__restrict__ v,
                                                      uint32_t nb, xdrg_status *status,
                                                      uint64_t *__restrict__ offsets, uint64_t n) {
  __shared__ unsigned long long part[1024];
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (nb + 1023u) / 1024u;
  const uint32_t a = min(nb, tid * per), b = min(nb, a + per);
  unsigned long long s = 0;
  for (uint32_t i = a; i < b; ++i) s += v[i];
  part[tid] = s;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    unsigned long long x = tid >= o ? part[tid - o] : 0ull;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  unsigned long long run = part[tid] - s;  // exclusive prefix of this thread's range
  for (uint32_t i = a; i < b; ++i) {
    const unsigned long long x = v[i];
    v[i] = run;
    run += x;
  }
  if (tid == 1023) {
    status->total_bytes = part[1023];
    offsets[n] = part[1023];
  }
}

// ------------------------------------------------------------ var: encode
__global__ __launch_bounds__(256) void k_var_encode(
    const uint8_t *__restrict__ native, uint64_t n, uint32_t stride, const uint8_t *__restrict__ heap,
    uint64_t heap_len, uint8_t *__restrict__ xdr, uint64_t cap, uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ sizes, const unsigned long long *__restrict__ block_base,
    const xdrg_op *__restrict__ ops, uint32_t nops, const uint32_t *__restrict__ table,
    uint32_t stack_limit, unsigned long long *err) {
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
  unsigned long long wbase = 0;
  for (uint32_t w = 0; w < wid; ++w) wbase += wsum[w];
  const uint64_t off = block_base[blockIdx.x] + wbase + incl - v;
  if (r >= n) return;
  offsets[r] = off;
  if (sz & kSizeErr) return;  // size pass reported this record

  const uint8_t *nat = native + r * stride;
  uint64_t pos = off;
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
    default: ++pc; break;
    }
  }
}

// ------------------------------------------------------------ var: decode
// Record r = xdr_from_opaque(stream[off[r], off[r+1]), r): fields walk in
// plan order with check() before every read; payloads go to the heap at
// [off[r], ...) 4-byte aligned; the native record is zero-filled first.
__global__ __launch_bounds__(256) void k_var_decode(
    const uint8_t *__restrict__ xdr, uint64_t len, const uint64_t *__restrict__ offsets, uint64_t n,
    uint8_t *__restrict__ native, uint32_t stride, uint8_t *__restrict__ heap,
    const xdrg_op *__restrict__ ops, uint32_t nops, const uint32_t *__restrict__ table,
    uint32_t stack_limit, unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  xdrg_op *sops = reinterpret_cast<xdrg_op *>(smem);
  load_ops(sops, ops, nops);
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint64_t a = offsets[r], b = offsets[r + 1];
  if (r == n - 1 && b != len) report(err, n, kOpRecordLevel, XDRG_ERR_TRAILING);
  if (b < a || b > len) { report(err, r, 0, XDRG_ERR_OVERFLOW_GET); return; }
  if ((b - a) & 3u) { report(err, r, kOpRecordLevel, XDRG_ERR_SIZE_NOT_MULT4); return; }
  uint8_t *nat = native + r * stride;
  for (uint32_t k = 0; k < stride / 4; ++k) st32(nat + 4 * k, 0u);
  uint64_t p = a, hcur = a;
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
      for (uint32_t k = 0; k < nw; ++k) st32(heap + hcur + 4ull * k, ld32(xdr + p + 4ull * k));
      if (L & 3u) {
        const uint32_t w = ld32(xdr + p + 4ull * (nw - 1));
        if (w & ~keep_mask(L & 3u)) { report(err, r, pc, XDRG_ERR_NONZERO_PAD); return; }
      }
      *reinterpret_cast<uint64_t *>(nat + op.noff) = hcur;
      st32(nat + op.noff + 8, L);
      hcur += 4ull * nw;
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
    default: ++pc; break;
    }
  }
  if (p != b) report(err, r, kOpRecordLevel, XDRG_ERR_TRAILING);
  return;
overflow:
  report(err, r, pc, XDRG_ERR_OVERFLOW_GET);
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
int run_fixed(const xdrg_plan &p, bool decode, const void *in, void *out, uint64_t nrec,
              unsigned long long *err, hipStream_t s) {
  if (nrec == 0) return XDRG_OK;
  const fixed_prog &pg = decode ? p.dec : p.enc;
  const bool checks = decode && p.has_checks;
  if (p.path == XDRG_PATH_FIXED_REG && aligned(in, 16) && aligned(out, 16)) {
    // Launch shapes from tools/tune/tune_fixed.py (rec128):
    //  * working set (input + output) that fits the 256 MiB Infinity Cache
    //    (1M records = 256 MiB): plain 16-byte loads/stores, one chunk in
    //    flight per lane, 1024 workgroups -> 6.9 TB/s back to back;
    //  * larger batches stream from HBM: non-temporal loads/stores, two
    //    chunks in flight per lane, 512 workgroups -> 5.76 TB/s at 16M
    //    records (a plain 16-byte copy of the same bytes: 5.67 TB/s).
    const uint32_t W = p.fixed_size;
    const uint32_t cpr = W / 16;
    const uint64_t nchunks = nrec * cpr;
    const bool streaming = nchunks * 32ull > kMallBytes * 3 / 2;  // in+out bytes > 384 MiB
    uint64_t blocks = (nchunks + 255) / 256;
    blocks = std::min<uint64_t>(blocks, streaming ? 512 : 1024);
    const uint32_t g0 = cpr / gcd32(cpr, 256);
    blocks = align_up(std::max<uint64_t>(blocks, 1), g0);
    const reg_word *prog = decode ? p.d_dec_reg : p.d_enc_reg;
    const bool bools = pg.has_bool;
    const u32x4 *i4 = static_cast<const u32x4 *>(in);
    u32x4 *o4 = static_cast<u32x4 *>(out);
#define LAUNCH_REG(B, C)                                                                         \
  do {                                                                                           \
    if (streaming)                                                                               \
      k_fixed_reg<B, C, 2, true><<<blocks, 256, 0, s>>>(i4, o4, nchunks, cpr, prog, p.d_table, err); \
    else                                                                                         \
      k_fixed_reg<B, C, 1, false><<<blocks, 256, 0, s>>>(i4, o4, nchunks, cpr, prog, p.d_table, err); \
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
  const uint32_t in_words = pg.in_words, out_words = pg.out_words;
  if (in_words > 8192) return XDRG_EUNSUPPORTED;  // > 32 KiB records: tile won't fit
  uint32_t T = std::min<uint32_t>(256, std::max<uint32_t>(4, 8192 / in_words));
  T &= ~3u;
  const bool vec = aligned(in, 16) && aligned(out, 16) && (T * in_words) % 4 == 0 &&
                   (T * out_words) % 4 == 0;
  const size_t lds = 4ull * (T * in_words + 4) + 4ull * ((out_words + 3u) & ~3u) +
                     sizeof(term) * pg.terms.size();
  const uint64_t tiles = (nrec + T - 1) / T;
  const uint64_t blocks = std::min<uint64_t>(tiles, 4096);
  const term_idx *idx = decode ? p.d_dec_idx : p.d_enc_idx;
  const term *terms = decode ? p.d_dec_terms : p.d_enc_terms;
  const uint32_t nterms = uint32_t(pg.terms.size());
  const uint32_t nchecks = checks ? uint32_t(p.checks.size()) : 0u;
  auto *i32 = static_cast<const uint32_t *>(in);
  auto *o32 = static_cast<uint32_t *>(out);
#define LAUNCH_LDS(C, V)                                                                   \
  k_fixed_lds<C, V><<<blocks, 256, lds, s>>>(i32, o32, nrec, in_words, out_words, T, idx, \
                                             terms, nterms, p.d_checks, nchecks, p.d_table, err)
  if (checks) {
    if (vec) LAUNCH_LDS(true, true); else LAUNCH_LDS(true, false);
  } else {
    if (vec) LAUNCH_LDS(false, true); else LAUNCH_LDS(false, false);
  }
#undef LAUNCH_LDS
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

size_t var_ws_layout(uint64_t n, size_t *sizes_off, size_t *bsum_off) {
  const uint64_t nb = (n + 255) / 256;
  *sizes_off = 0;
  *bsum_off = align_up(n * 4, 256);
  return *bsum_off + align_up(nb * 8, 256);
}

unsigned long long *err_ptr(xdrg_status *st) {
  return reinterpret_cast<unsigned long long *>(&st->first_error);
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
  xdrg_plan *p = new (std::nothrow) xdrg_plan();
  if (!p) return XDRG_ENOMEM;
  p->ops.assign(ops, ops + nops);
  if (ntable) p->table.assign(table, table + ntable);
  p->stride = native_stride;
  int rc = xdrg::compile_plan(*p);
  if (rc != XDRG_OK) { delete p; return rc; }
  if (p->stride % 4) { delete p; return XDRG_EUNSUPPORTED; }
  // One device allocation holding every table.
  struct part { const void *src; size_t bytes; size_t off; };
  part parts[10] = {
      {p->ops.data(), p->ops.size() * sizeof(xdrg_op), 0},
      {p->table.data(), p->table.size() * 4, 0},
      {p->enc.idx.data(), p->enc.idx.size() * sizeof(term_idx), 0},
      {p->enc.terms.data(), p->enc.terms.size() * sizeof(term), 0},
      {p->dec.idx.data(), p->dec.idx.size() * sizeof(term_idx), 0},
      {p->dec.terms.data(), p->dec.terms.size() * sizeof(term), 0},
      {p->enc.reg.data(), p->enc.reg.size() * sizeof(reg_word), 0},
      {p->dec.reg.data(), p->dec.reg.size() * sizeof(reg_word), 0},
      {p->checks.data(), p->checks.size() * sizeof(check), 0},
      {nullptr, 16, 0}};
  size_t total = 0;
  for (part &q : parts) { q.off = total; total += align_up(q.bytes, 256); }
  hipError_t e = hipMalloc(&p->d_mem, total);
  if (e != hipSuccess) { delete p; return hip_fail(e, "hipMalloc(plan)"); }
  char *base = static_cast<char *>(p->d_mem);
  for (part &q : parts)
    if (q.src && q.bytes) {
      e = hipMemcpy(base + q.off, q.src, q.bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) { (void)hipFree(p->d_mem); delete p; return hip_fail(e, "hipMemcpy(plan)"); }
    }
  p->d_ops = reinterpret_cast<const xdrg_op *>(base + parts[0].off);
  p->d_table = reinterpret_cast<const uint32_t *>(base + parts[1].off);
  p->d_enc_idx = reinterpret_cast<const term_idx *>(base + parts[2].off);
  p->d_enc_terms = reinterpret_cast<const term *>(base + parts[3].off);
  p->d_dec_idx = reinterpret_cast<const term_idx *>(base + parts[4].off);
  p->d_dec_terms = reinterpret_cast<const term *>(base + parts[5].off);
  p->d_enc_reg = reinterpret_cast<const reg_word *>(base + parts[6].off);
  p->d_dec_reg = reinterpret_cast<const reg_word *>(base + parts[7].off);
  p->d_checks = reinterpret_cast<const check *>(base + parts[8].off);
  *out = p;
  return XDRG_OK;
}

void xdrg_plan_destroy(xdrg_plan *p) {
  if (!p) return;
  if (p->d_mem) (void)hipFree(p->d_mem);
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
  return XDRG_OK;
}

size_t xdrg_workspace_size(const xdrg_plan *p, uint64_t n) {
  if (!p || p->path != XDRG_PATH_VAR) return 0;
  size_t a, b;
  return var_ws_layout(n, &a, &b);
}

int xdrg_status_init(xdrg_status *st, void *stream) {
  if (!st) return XDRG_EINVAL;
  HIPCHK(hipMemsetAsync(st, 0xff, 8, static_cast<hipStream_t>(stream)));
  HIPCHK(hipMemsetAsync(reinterpret_cast<char *>(st) + 8, 0, 8, static_cast<hipStream_t>(stream)));
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
    return run_fixed(*p, false, d_native, d_xdr, nrec, err, s);
  }
  // ---- variable plans
  if (!d_offsets) return XDRG_EINVAL;
  if (d_heap && !aligned(d_heap, 4)) return XDRG_EALIGN;
  if (!aligned(d_native, 8) || !aligned(d_xdr, 4) || !aligned(d_offsets, 8)) return XDRG_EALIGN;
  if (n == 0) {
    HIPCHK(hipMemsetAsync(d_offsets, 0, 8, s));
    return XDRG_OK;
  }
  size_t so, bo;
  const size_t need = var_ws_layout(n, &so, &bo);
  if (!d_ws || ws_bytes < need) return XDRG_ESPACE;
  uint32_t *sizes = reinterpret_cast<uint32_t *>(static_cast<char *>(d_ws) + so);
  unsigned long long *bsum = reinterpret_cast<unsigned long long *>(static_cast<char *>(d_ws) + bo);
  const uint64_t nb = (n + 255) / 256;
  if (nb > 0xffffffffull) return XDRG_EUNSUPPORTED;
  const size_t lds_ops = p->ops.size() * sizeof(xdrg_op);
  k_var_size<<<nb, 256, lds_ops, s>>>(static_cast<const uint8_t *>(d_native), n, p->stride,
                                       p->d_ops, uint32_t(p->ops.size()), p->d_table, sizes,
                                       bsum, err);
  HIPCHK(hipGetLastError());
  k_scan_blocks<<<1, 1024, 0, s>>>(bsum, uint32_t(nb), d_status, d_offsets, n);
  HIPCHK(hipGetLastError());
  k_var_encode<<<nb, 256, lds_ops, s>>>(static_cast<const uint8_t *>(d_native), n, p->stride,
                                         d_heap, heap_len, static_cast<uint8_t *>(d_xdr), cap,
                                         d_offsets, sizes, bsum, p->d_ops,
                                         uint32_t(p->ops.size()), p->d_table, stack_limit, err);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

int xdrg_decode(const xdrg_plan *p, const void *d_xdr, uint64_t len, const uint64_t *d_offsets,
                uint64_t n, void *d_native, uint8_t *d_heap_out, uint64_t heap_cap,
                uint32_t stack_limit, void *d_ws, size_t ws_bytes, xdrg_status *d_status,
                void *stream) {
  (void)d_ws;
  (void)ws_bytes;
  if (!p || !d_status || (n && (!d_native || (len && !d_xdr)))) return XDRG_EINVAL;
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
    return run_fixed(*p, true, d_xdr, d_native, nrec, err, s);
  }
  if (!d_offsets) return XDRG_EUNSUPPORTED;  // var decode needs a record index
  if (n == 0) {
    if (len) return launch_report(err, 0, kOpRecordLevel, XDRG_ERR_TRAILING, s);
    return XDRG_OK;
  }
  if (heap_cap < len || (len && !d_heap_out)) return XDRG_ESPACE;
  if (!aligned(d_xdr, 4) || !aligned(d_native, 8) || (d_heap_out && !aligned(d_heap_out, 4)))
    return XDRG_EALIGN;
  const uint64_t nb = (n + 255) / 256;
  const size_t lds_ops = p->ops.size() * sizeof(xdrg_op);
  k_var_decode<<<nb, 256, lds_ops, s>>>(static_cast<const uint8_t *>(d_xdr), len, d_offsets, n,
                                         static_cast<uint8_t *>(d_native), p->stride, d_heap_out,
                                         p->d_ops, uint32_t(p->ops.size()), p->d_table,
                                         stack_limit, err);
  HIPCHK(hipGetLastError());
  return XDRG_OK;
}

int xdrg_serial_sizes(const xdrg_plan *p, const void *d_native, uint64_t n, uint32_t *d_sizes,
                      uint32_t stack_limit, xdrg_status *d_status, void *stream) {
  if (!p || !d_status || (n && (!d_native || !d_sizes))) return XDRG_EINVAL;
  if (n == 0) return XDRG_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p->path != XDRG_PATH_VAR) {
    // fixed_size for every record (xdr_struct_base_fs, types.h:691-700)
    HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_sizes), int(p->fixed_size), n, s));
    return XDRG_OK;
  }
  const uint64_t nb = (n + 255) / 256;
  unsigned long long *bsum = nullptr;
  HIPCHK(hipMallocAsync(reinterpret_cast<void **>(&bsum), nb * 8, s));
  k_var_size<<<nb, 256, p->ops.size() * sizeof(xdrg_op), s>>>(
      static_cast<const uint8_t *>(d_native), n, p->stride, p->d_ops, uint32_t(p->ops.size()),
      p->d_table, d_sizes, bsum, err_ptr(d_status));
  HIPCHK(hipGetLastError());
  HIPCHK(hipFreeAsync(bsum, s));
  return XDRG_OK;
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
  default: return "unknown xdrgpu error";
  }
}

int xdrg_error_exception(int code) {
  switch (code) {
  case XDRG_ERR_OVERFLOW_GET: case XDRG_ERR_OVERFLOW_PUT: case XDRG_ERR_XVECTOR_BOUND:
  case XDRG_ERR_XSTRING_BOUND: return XDRG_EXC_OVERFLOW;
  case XDRG_ERR_NONZERO_PAD: return XDRG_EXC_SHOULD_BE_ZERO;
  case XDRG_ERR_BAD_DISCRIMINANT: return XDRG_EXC_BAD_DISCRIMINANT;
  case XDRG_ERR_INVALID_ENUM: return XDRG_EXC_INVARIANT_FAILED;
  case XDRG_ERR_STACK_PUT: case XDRG_ERR_STACK_GET: return XDRG_EXC_STACK_OVERFLOW;
  case XDRG_ERR_SIZE_NOT_MULT4: case XDRG_ERR_TRAILING: return XDRG_EXC_BAD_MESSAGE_SIZE;
  default: return XDRG_EXC_NONE;
  }
}

}  // extern "C"
