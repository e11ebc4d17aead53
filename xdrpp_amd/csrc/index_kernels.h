// The segment pass of the stream indexes (xdrg_index_msgs,
// xdrg_index_records): shared by the library (xdrgpu.hip) and the
// plan-specialized kernels (spec.cpp: a generated record parse), so it
// compiles under hiprtc too.  The rest of the list ranking (k_ix_up,
// k_ix_down, k_ix_emit) and the interpreted parse stay in xdrgpu.hip.
#pragma once
#include "dev_common.h"

namespace xdrg {
namespace dev {

constexpr uint32_t kIxSW = 4096;  // words per segment (16 KiB)
constexpr uint32_t kIxLog = 12;   // log2(kIxSW) pointer-jumping rounds
constexpr uint64_t kIxCnt = (1ull << 40) - 1;  // table / entry word: count bits

// Record parse results: RX_BAD (not a record start the decode accepts),
// RX_LONG (runs past the index window, not past the stream).
constexpr uint32_t RX_BAD = 0xffffffffu, RX_LONG = 0xfffffffeu;

// 16 words of a segment per thread (4 x 16 bytes, all in flight at once):
// raw[4g + j] = word 4 * (tid + 256 g) + j of the segment (0 past the stream).
__device__ __forceinline__ void ix_load16(const uint8_t *__restrict__ s, uint64_t len, uint64_t w0,
                                          uint32_t tid, uint32_t raw[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const uint64_t w = w0 + 4u * (tid + 256u * g);
    if (4 * w + 16 <= len) {
      const u32x4 q = ld16u(s + 4 * w);
      raw[4 * g] = q.x; raw[4 * g + 1] = q.y; raw[4 * g + 2] = q.z; raw[4 * g + 3] = q.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) raw[4 * g + j] = 4 * (w + j) + 4 <= len ? ld32(s + 4 * (w + j)) : 0u;
    }
  }
}

// Valid-node test with segment-local 32-bit arithmetic: node i of a segment
// whose stream bytes end `lim` bytes after its start (lim >= 4 * i).  A
// valid mark's first two bytes are 0x80 0x00 (last-fragment bit, size <
// 2^16 and the pre-swap size test passes), so one compare rejects almost
// every other word.  Returns the next mark's node index (may be past the
// segment) or 0xffffffff when a chain reaching node i ends there.
__device__ __forceinline__ uint32_t ix_next(uint32_t raw, uint32_t i, uint32_t lim, uint32_t maxlen) {
  const uint32_t at = 4u * i;
  if ((raw & 0xffffu) != 0x80u || lim - at < 4u) return 0xffffffffu;
  const uint32_t size = ((raw >> 8) & 0xff00u) | (raw >> 24);
  if (size > maxlen || (size & 3u) || lim - at - 4u < size) return 0xffffffffu;
  return i + 1u + size / 4u;
}

// LDS node: target (13 bits: < kIxSW a node of this segment, kIxSW + e =
// entry e of the next one) | marks passed << 13 (13 bits) | ends << 26.
// Table word: marks (40 bits) | exit entry << 40 (16 bits) | ends << 56.
// List word of a valid node: node index | target << 12.
constexpr uint32_t kIxEnds = 1u << 26;


// REC: record starts (xdrg_index_records): P parses a record from a byte
// offset (the library's interpreted rx_len, or a plan's generated parse);
// otherwise record marks (xdrg_index_msgs).  has_first / fd: the first
// checked word of a record and its byte offset (P::first_ok tests it).
template <bool REC, class P>
__device__ __forceinline__ void ix_seg_body(const P &parser, const uint8_t *__restrict__ s, uint64_t len,
                                            uint32_t maxlen, uint32_t K, uint64_t *__restrict__ tab,
                                            uint32_t *__restrict__ list, uint32_t *__restrict__ lcount,
                                            bool has_first, uint32_t fd) {
  __shared__ __attribute__((aligned(16))) uint32_t node[kIxSW];
  __shared__ uint16_t lst[kIxSW];
  __shared__ uint32_t wtot[4];
  extern __shared__ __attribute__((aligned(16))) uint32_t rx_smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  const uint64_t w0 = static_cast<uint64_t>(blockIdx.x) * kIxSW;
  const uint32_t lim = static_cast<uint32_t>(min<uint64_t>(len - 4 * w0, 0xfffffff0ull));
  uint32_t raw[16];
  if (REC) parser.init(rx_smem);
  else ix_load16(s, len, w0, tid, raw);
  // REC: the first checked word of every candidate start, all in flight
  // at once; only starts that pass it are walked
  uint32_t first[16];
  if (REC) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint64_t a = 4 * (w0 + 4u * (tid + 256u * (q >> 2)) + (q & 3));
      first[q] = !has_first || a + fd + 4 > len ? 0u : ld32(s + a + fd);
    }
  }
  // REC: the wave's candidates that pass their first word are walked as one
  // queue (64 lanes per round, lst holds the wave's queue: 1024 entries), not
  // candidate slot by candidate slot -- a slot where a few lanes pass would
  // otherwise walk with the rest idle.  A walk leaves its successor in
  // node[i]; the owner lane reads it back below.
  uint32_t pmask = 0;
  if (REC) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t i = 4u * (tid + 256u * (q >> 2)) + (q & 3);
      const uint64_t a = 4 * (w0 + i);
      const bool cand = a < len && (!has_first || (a + fd + 4 <= len && fd + 4 <= maxlen &&
                                                   parser.first_ok(rx_smem, bswap32(first[q]))));
      if (cand) pmask |= 1u << q;
    }
    const uint32_t pc = __popc(pmask);
    uint32_t pin = pc;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(pin, o, 64);
      if (lane >= static_cast<uint32_t>(o)) pin += y;
    }
    const uint32_t ptot = rl32(pin, 63);
    uint16_t *queue = lst + 1024u * wid;
    uint32_t qb = pin - pc;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (pmask & (1u << q)) queue[qb++] = static_cast<uint16_t>(4u * (tid + 256u * (q >> 2)) + (q & 3));
    wave_sync();
    for (uint32_t k = lane; k < ptot; k += 64u) {
      const uint32_t i = queue[k];
      const uint32_t L = parser.rlen(rx_smem, s, len, 4 * (w0 + i), maxlen);
      node[i] = L < RX_LONG ? i + L / 4u : 0xffffffffu;
    }
    wave_sync();
  }
  uint32_t vmask = 0, vnext[16];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint32_t nv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = 4 * g + j;
      const uint32_t i = 4u * (tid + 256u * g) + j;
      if (REC) {
        vnext[q] = (pmask & (1u << q)) ? node[i] : 0xffffffffu;
      } else {
        vnext[q] = ix_next(raw[q], i, lim, maxlen);
      }
      if (vnext[q] != 0xffffffffu) vmask |= 1u << q;
      nv[j] = vnext[q] != 0xffffffffu ? (vnext[q] | (1u << 13)) : kIxEnds;
    }
    reinterpret_cast<u32x4 *>(node)[tid + 256u * g] = u32x4{nv[0], nv[1], nv[2], nv[3]};
  }
  // compact the valid nodes: block-wide exclusive scan of the counts
  const uint32_t cnt = __popc(vmask);
  uint32_t incl = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= static_cast<uint32_t>(o)) incl += y;
  }
  if (lane == 63) wtot[wid] = incl;
  __syncthreads();
  uint32_t base = incl - cnt, nvalid = 0;
  for (uint32_t w = 0; w < 4; ++w) {
    if (w < wid) base += wtot[w];
    nvalid += wtot[w];
  }
  uint32_t *gl = list + static_cast<uint64_t>(blockIdx.x) * kIxSW;
#pragma unroll
  for (int q = 0; q < 16; ++q)
    if (vmask & (1u << q)) {
      const uint32_t i = 4u * (tid + 256u * (q >> 2)) + (q & 3);
      lst[base] = static_cast<uint16_t>(i);
      gl[base] = i | (vnext[q] << 12);
      ++base;
    }
  if (tid == 0) lcount[blockIdx.x] = nvalid;
  __syncthreads();
  // Pointer jumping over the valid nodes, in place: a node read mid-round
  // is either state, each a correct jump.  Stops once no valid node points
  // inside the segment.
  for (uint32_t k = 0; k < kIxLog + 1; ++k) {
    bool inside = false;
    for (uint32_t j = tid; j < nvalid; j += 256) {
      const uint32_t i = lst[j];
      const uint32_t v = node[i];
      const uint32_t t = v & 0x1fffu;
      if (!(v & kIxEnds) && t < kIxSW) {
        const uint32_t u = node[t];
        const uint32_t c = ((v >> 13) & 0x1fffu) + ((u >> 13) & 0x1fffu);
        const uint32_t nv = (u & ~(0x1fffu << 13)) | (c << 13);
        node[i] = nv;
        inside |= !(nv & kIxEnds) && (nv & 0x1fffu) < kIxSW;
      }
    }
    if (!__syncthreads_or(inside)) break;
  }
  if (!tab) return;
  for (uint32_t e = tid; e < K; e += 256) {
    const uint32_t v = node[e];
    const uint64_t c = (v >> 13) & 0x1fffu;
    tab[static_cast<uint64_t>(blockIdx.x) * K + e] =
        (v & kIxEnds) ? (1ull << 56 | c) : (static_cast<uint64_t>((v & 0x1fffu) - kIxSW) << 40 | c);
  }
}


}  // namespace dev
}  // namespace xdrg
