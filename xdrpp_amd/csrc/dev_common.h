// Device helpers shared by the library's kernels (xdrgpu.hip, rpc.hip) and
// by the plan-specialized kernels compiled at plan time (hiprtc, see
// spec.cpp): byte swaps, error reports, unaligned and clamped loads, LDS
// staging, record marks, cross-lane reads.  Self-contained so hiprtc can
// compile it (no C++ standard headers).
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include "xdrgpu.h"

namespace xdrg {
namespace dev {

constexpr uint32_t kOpRecordLevel = 0xffff;  // op field for record-level errors
constexpr uint32_t kSizeErr = 0x80000000u;  // size-pass marker of a failed record

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// D = bytes of {hi:lo} picked by sel (v_perm_b32): 0-3 from lo, 4-7 from hi,
// 0x0C -> 0x00.
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// The lowest failing (record, op) wins: the record at which the
// reference's sequential archive would have thrown.
__device__ __forceinline__ void report(unsigned long long *err, uint64_t rec, uint32_t op,
                                       uint32_t code) {
  const unsigned long long key =
      (static_cast<unsigned long long>(rec) << 24) |
      (static_cast<unsigned long long>(op & 0xffffu) << 8) | code;
  atomicMin(err, key);
}

// Uniform trip count, no per-lane exit: the table reads stay scalar.
__device__ __forceinline__ bool enum_ok(const uint32_t *__restrict__ table, uint32_t idx,
                                        uint32_t cnt, uint32_t v) {
  bool ok = false;
  for (uint32_t i = 0; i < cnt; ++i) ok |= table[idx + i] == v;
  return ok;
}

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
// Decode: the element area of one container of `cnt` inline elements of
// `stride` native and `wire` wire bytes, `rem` wire bytes left after its
// count.  Aligns the bump pointer to 8 and checks that the elements the
// bytes left can reach (the ones before the first that runs out, and that
// one) fit before `eend`.  Valid data always fits (the heap factor,
// xdrg_decode_heap_size); a forged count in a truncated record fails here
// with xdr_overflow, the error the reference raises at the element that
// runs out, instead of writing past the record's area.
__device__ __forceinline__ bool elem_area_ok(uint64_t &ecur, uint64_t eend, uint32_t cnt, uint32_t stride,
                                             uint32_t wire, uint64_t rem) {
  ecur = (ecur + 7u) & ~7ull;
  const uint64_t reach = min(static_cast<uint64_t>(cnt), rem / wire + 1) * stride;
  return ecur <= eend && reach <= eend - ecur;
}
__device__ __forceinline__ uint32_t keep_mask(uint32_t nbytes) {  // nbytes in 1..4
  return nbytes >= 4 ? 0xffffffffu : ((1u << (8u * nbytes)) - 1u);
}
__device__ __forceinline__ uint32_t keep_bytes(int32_t k) {  // mask of the low k bytes, k clamped
  return k <= 0 ? 0u : k >= 4 ? 0xffffffffu : ((1u << (8 * k)) - 1u);
}

// Unaligned 16-byte global access: correct at any byte alignment on gfx950
// (tools/probe/unaligned.hip).
__device__ __forceinline__ u32x4 ld16u(const uint8_t *p) { return *reinterpret_cast<const u32x4 *>(p); }
__device__ __forceinline__ void st16u(uint8_t *p, u32x4 v) { *reinterpret_cast<u32x4 *>(p) = v; }

// Single-wave workgroups: LDS written by some lanes and read by others needs
// only ordering within the wave (LDS executes a wave's instructions in
// order), not __syncthreads(), whose workgroup-scope release would also
// wait for every outstanding global store of the wave (s_waitcnt vmcnt(0)).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Stage nbytes (a multiple of 4) of native records from a 16-byte aligned
// global address to LDS: 16-byte loads, up to UL per lane in flight before
// any LDS store (one memory round trip per UL KiB per 64 threads).
template <int UL = 4>
__device__ __forceinline__ void stage_tile(uint8_t *tile, const uint8_t *src, uint32_t nbytes,
                                           uint32_t lane, uint32_t nthreads) {
  const uint32_t n16 = nbytes / 16u;
  for (uint32_t i0 = 0; i0 < n16; i0 += UL * nthreads) {
    u32x4 t[UL];
#pragma unroll
    for (int k = 0; k < UL; ++k) {
      const uint32_t i = i0 + k * nthreads + lane;
      if (i < n16) t[k] = reinterpret_cast<const u32x4 *>(src)[i];
    }
#pragma unroll
    for (int k = 0; k < UL; ++k) {
      const uint32_t i = i0 + k * nthreads + lane;
      if (i < n16) reinterpret_cast<u32x4 *>(tile)[i] = t[k];
    }
  }
  for (uint32_t i = n16 * 4u + lane; i < nbytes / 4u; i += nthreads)
    reinterpret_cast<uint32_t *>(tile)[i] = reinterpret_cast<const uint32_t *>(src)[i];
}

// ------------------------------------------- record marks (RFC 5531)
// message_t keeps a 4-byte mark BE(size | 0x80000000) in front of the
// message bytes (message_t::alloc, xdrpp/marshal.cc:15-31: always one
// last-fragment record).
__device__ __forceinline__ uint32_t mark_word(uint32_t size) { return bswap32(size | XDRG_MARK_LAST); }

// Framing checks of a message whose record index gives it `body` bytes
// after the mark, in read_message's order (xdrpp/srpc.cc:29-55).  The
// first test reads the mark before swap32le, so on a little-endian host it
// looks at the low bits of the mark's first byte (bits 24-25 of the size),
// which is what the reference does on this platform.  0 = well framed.
__device__ __forceinline__ uint32_t mark_code(uint32_t raw, uint64_t body) {
  if (raw & 3u) return XDRG_ERR_MSG_SIZE4;          // srpc.cc:38-39
  const uint32_t v = bswap32(raw);
  if (!(v & XDRG_MARK_LAST)) return XDRG_ERR_MSG_FRAGMENT;  // srpc.cc:41-45
  if ((v & ~XDRG_MARK_LAST) != body) return XDRG_ERR_MSG_MISMATCH;
  return 0u;
}

// Registers of one lane read by the whole wave (v_readlane).
__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t lane) {
  return __builtin_amdgcn_readlane(v, lane);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t lane) {
  return static_cast<uint64_t>(rl32(static_cast<uint32_t>(v), lane)) |
         (static_cast<uint64_t>(rl32(static_cast<uint32_t>(v >> 32), lane)) << 32);
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP moves (no LDS
// round trip, unlike __shfl_up's ds_bpermute): row_shr 1/2/4/8 scans each
// row of 16 lanes, row_bcast:15 and row_bcast:31 carry row totals into the
// rows above.  Every lane of the wave must be active.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x) {
  return x + static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), CTRL, ROWS, 0xf, true));
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x = dpp_add<0x111, 0xf>(x);  // row_shr:1
  x = dpp_add<0x112, 0xf>(x);  // row_shr:2
  x = dpp_add<0x114, 0xf>(x);  // row_shr:4
  x = dpp_add<0x118, 0xf>(x);  // row_shr:8
  x = dpp_add<0x142, 0xa>(x);  // row_bcast:15 -> rows 1, 3
  x = dpp_add<0x143, 0xc>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Packed element areas (plans with no recursive type; oracle/
// xdr_oracle.c rec_ebytes): the wave's 64 records are one group, whose
// arrays follow each other from align8(ebase + F * a of the first record).
// E = the record's share (the walker's ebytes, capped at
// align8-down(F * (b - a) - 8)); `bad` = offsets the decode refuses (b < a,
// b > len).  From the first bad record on the group gets empty areas: the
// records before it lie inside [a0, b) of the stream, so their shares stay
// inside the group's F-sized area whatever the later offsets hold, and the
// reported error is that record's (or an earlier one's).  Every lane of the
// wave must be active.
__device__ __forceinline__ uint64_t ebudget(uint32_t F, uint64_t a, uint64_t b) {
  const uint64_t t = static_cast<uint64_t>(F) * (b - a);
  return t >= 8u ? (t - 8u) & ~7ull : 0u;
}
__device__ __forceinline__ uint64_t packed_area(uint64_t E, bool bad, uint64_t a0, uint64_t ebase, uint32_t F,
                                                uint64_t &ecur, uint64_t &eend) {
  const uint32_t lane = __lane_id();
  const unsigned long long bm = __ballot(bad);
  if (bm & ((2ull << lane) - 1ull)) E = 0;  // a bad record at or before this one
  uint64_t inc = E;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t x = __shfl_up(inc, o, 64);
    if (lane >= static_cast<uint32_t>(o)) inc += x;
  }
  const uint64_t g0 = (ebase + static_cast<uint64_t>(F) * a0 + 7u) & ~7ull;
  ecur = g0 + inc - E;
  eend = g0 + inc;
  return g0;
}

}  // namespace dev
}  // namespace xdrg
