// Device helpers and the fixed-size kernels (k_fixed_reg / k_fixed_lds).
// Included by xdrgpu.hip (the product library) and by the tuning harness
// under tools/tune/, which sweeps the template parameters.
#pragma once
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "plan.h"

namespace xdrg {
namespace dev {

// xdr_traits<bool> (xdrpp/types.h:335-349).  sel: src byte | dst byte << 8 |
// whole-word test << 16.
__device__ __forceinline__ uint32_t bool_term(uint32_t v, uint32_t sel) {
  const bool nz = (sel & 0x10000u) ? (v != 0u) : (((v >> (8u * (sel & 3u))) & 0xffu) != 0u);
  return nz ? (1u << (8u * ((sel >> 8) & 3u))) : 0u;
}

// Decode-time word checks: padding of fixed opaque (marshal.cc:52-55) and
// opt-in enum validation (types.h:157-173).  Returns an xdrg_err or 0.
__device__ __forceinline__ uint32_t check_word(uint32_t w, uint32_t kind, uint32_t a, uint32_t b,
                                               const uint32_t *__restrict__ table) {
  if (kind == C_PAD) return (w & a) ? XDRG_ERR_NONZERO_PAD : 0u;
  if (kind == C_ENUM) return enum_ok(table, a, b, bswap32(w)) ? 0u : XDRG_ERR_INVALID_ENUM;
  return 0u;
}

__global__ void k_report(unsigned long long *err, uint64_t rec, uint32_t op, uint32_t code) {
  if (threadIdx.x == 0 && blockIdx.x == 0) report(err, rec, op, code);
}

// ---------------------------------------------------------- fixed: registers
// One lane = one 16-byte chunk per step.  The grid stride is a multiple of
// the chunks-per-record, so a lane's chunk position (and its program) never
// changes: selectors live in registers for the whole launch.
template <bool BOOLS, bool CHECKS, int U, bool NT = true>
__global__ __launch_bounds__(256) void k_fixed_reg(const u32x4 *__restrict__ in,
                                                   u32x4 *__restrict__ out, uint64_t nchunks,
                                                   uint32_t cpr, const reg_word *__restrict__ prog,
                                                   const uint32_t *__restrict__ table,
                                                   unsigned long long *err) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t q = static_cast<uint32_t>(c0 % cpr);
  const reg_word *pw = prog + 4u * q;
  const uint32_t s0 = pw[0].sel, s1 = pw[1].sel, s2 = pw[2].sel, s3 = pw[3].sel;
  uint32_t k0 = T_PERM, k1 = T_PERM, k2 = T_PERM, k3 = T_PERM;
  if (BOOLS) { k0 = pw[0].kind; k1 = pw[1].kind; k2 = pw[2].kind; k3 = pw[3].kind; }
  uint32_t ck[4] = {0, 0, 0, 0}, cop[4] = {0, 0, 0, 0}, ca[4] = {0, 0, 0, 0}, cb[4] = {0, 0, 0, 0};
  if (CHECKS) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ck[i] = pw[i].ck_kind; cop[i] = pw[i].ck_op; ca[i] = pw[i].ck_a; cb[i] = pw[i].ck_b;
    }
  }
  for (uint64_t c = c0; c < nchunks; c += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t cc = c + u * stride;
      if (cc < nchunks) v[u] = NT ? __builtin_nontemporal_load(in + cc) : in[cc];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t cc = c + u * stride;
      if (cc < nchunks) {
        const u32x4 w = v[u];
        u32x4 o;
        o.x = perm(w.y, w.x, s0);
        o.y = perm(w.y, w.x, s1);
        o.z = perm(w.w, w.z, s2);
        o.w = perm(w.w, w.z, s3);
        if (BOOLS) {
          if (k0 == T_BOOL) o.x = bool_term(w.x, s0);
          if (k1 == T_BOOL) o.y = bool_term(w.y, s1);
          if (k2 == T_BOOL) o.z = bool_term(w.z, s2);
          if (k3 == T_BOOL) o.w = bool_term(w.w, s3);
        }
        if (CHECKS) {
          const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (ck[i]) {
              const uint32_t e = check_word(wv[i], ck[i], ca[i], cb[i], table);
              if (e) report(err, cc / cpr, cop[i], e);
            }
        }
        if (NT) __builtin_nontemporal_store(o, out + cc); else out[cc] = o;
      }
    }
  }
}

// -------------------------------------------------------------- fixed: LDS
// A workgroup processes tiles of T records: coalesced load of T input
// records into LDS, optional validation of the staged wire words, then each
// lane builds 4 consecutive output words from the term program and stores
// them as one 16-byte write.
template <bool CHECKS, bool VEC>
__global__ __launch_bounds__(256) void k_fixed_lds(
    const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint64_t n, uint32_t in_words,
    uint32_t out_words, uint32_t T, const term_idx *__restrict__ g_idx,
    const term *__restrict__ g_terms, uint32_t nterms, const check *__restrict__ g_checks,
    uint32_t nchecks, const uint32_t *__restrict__ table, unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t *tile = smem;                         // T*in_words (+4 pad)
  const uint32_t tile_words = T * in_words + 4;  // multiple of 4 (T % 4 == 0)
  term_idx *sidx = reinterpret_cast<term_idx *>(smem + tile_words);
  term *sterms = reinterpret_cast<term *>(smem + tile_words + ((out_words + 3u) & ~3u));
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < out_words; i += blockDim.x) sidx[i] = g_idx[i];
  for (uint32_t i = tid; i < nterms; i += blockDim.x) sterms[i] = g_terms[i];
  if (tid < 4) tile[T * in_words + tid] = 0u;

  for (uint64_t t = blockIdx.x; t * T < n; t += gridDim.x) {
    const uint64_t r0 = t * T;
    const uint32_t nt = static_cast<uint32_t>(min<uint64_t>(T, n - r0));
    const uint32_t nin = nt * in_words;
    const uint32_t *src = in + r0 * in_words;
    __syncthreads();  // previous tile fully consumed (and table copies visible)
    if (VEC) {
      const uint32_t nv = nin >> 2;
      const u32x4 *s4 = reinterpret_cast<const u32x4 *>(src);
      u32x4 *t4 = reinterpret_cast<u32x4 *>(tile);
      for (uint32_t i = tid; i < nv; i += blockDim.x) t4[i] = s4[i];
      for (uint32_t i = (nv << 2) + tid; i < nin; i += blockDim.x) tile[i] = src[i];
    } else {
      for (uint32_t i = tid; i < nin; i += blockDim.x) tile[i] = src[i];
    }
    __syncthreads();
    if (CHECKS) {
      for (uint32_t i = tid; i < nt * nchecks; i += blockDim.x) {
        const uint32_t r = i / nchecks, k = i - r * nchecks;
        const check ck = g_checks[k];
        const uint32_t e = check_word(tile[r * in_words + ck.word], ck.kind, ck.a, ck.b, table);
        if (e) report(err, r0 + r, ck.op, e);
      }
    }
    const uint32_t nout = nt * out_words;
    uint32_t *dst = out + r0 * out_words;
    for (uint32_t o4 = tid * 4u; o4 < nout; o4 += blockDim.x * 4u) {
      uint32_t r = o4 / out_words;
      uint32_t j = o4 - r * out_words;
      uint32_t vals[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t v = 0u;
        const term_idx ix = sidx[j];
        const uint32_t base = r * in_words;
        for (uint32_t q = 0; q < ix.count; ++q) {
          const term tm = sterms[ix.start + q];
          if (tm.kind == T_PERM)
            v |= perm(tile[base + tm.src + 1u], tile[base + tm.src], tm.sel);
          else
            v |= bool_term(tile[base + tm.src], tm.sel);
        }
        vals[i] = v;
        if (++j == out_words) { j = 0; ++r; }
      }
      if (VEC && o4 + 4u <= nout) {
        *reinterpret_cast<u32x4 *>(dst + o4) = u32x4{vals[0], vals[1], vals[2], vals[3]};
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (o4 + i < nout) dst[o4 + i] = vals[i];
      }
    }
  }
}


// ----------------------------------------------------------- fixed: group
// Non-identity fixed layouts (numerics: 56-byte native, 44-byte wire).  G
// records form a group whose input and output are whole 16-byte chunks; a
// lane owns output chunk position q of every group it visits (the grid
// stride is a multiple of the chunks per group), keeps its 4 x KT term
// program in registers, reads its terms' 8-byte windows straight from
// global memory (4-byte aligned dwordx2 loads; the wave's loads cover a
// contiguous stretch, so they coalesce in L1/L2), and stores one 16-byte
// chunk.  U chunks in flight per lane.  Full groups only; the host runs the
// tail (< G records) through k_fixed_lds.
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));

template <int KT, int U, bool NT = false>
__global__ __launch_bounds__(256) void k_fixed_grp(const uint8_t *__restrict__ in,
                                                   u32x4 *__restrict__ out, uint64_t nchunks,
                                                   uint32_t C, uint32_t in_g,
                                                   const grp_term *__restrict__ prog) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t q = static_cast<uint32_t>(c0 % C);
  const uint64_t gstep = stride / C;
  uint32_t off[4][KT], sel[4][KT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const grp_term t = prog[(q * 4u + i) * KT + k];
      off[i][k] = t.off;
      sel[i][k] = t.sel;
    }
  uint64_t g = c0 / C;
  for (uint64_t c = c0; c < nchunks; c += U * stride, g += U * gstep) {
    u32x2a w[U][4][KT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint8_t *base = in + (g + u * gstep) * in_g;
      if (c + u * stride < nchunks) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int k = 0; k < KT; ++k)
            w[u][i][k] = *reinterpret_cast<const u32x2a *>(base + off[i][k]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t cc = c + u * stride;
      if (cc < nchunks) {
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint32_t v = 0;
#pragma unroll
          for (int k = 0; k < KT; ++k) {
            const uint32_t s = sel[i][k];
            const u32x2a x = w[u][i][k];
            if (s & kGrpBool)
              v |= bool_term((s & kGrpHi) ? x.y : x.x, s & 0xffffffu);
            else
              v |= perm(x.y, x.x, s);
          }
          o[i] = v;
        }
        const u32x4 ov = u32x4{o[0], o[1], o[2], o[3]};
        if (NT) __builtin_nontemporal_store(ov, out + cc); else out[cc] = ov;
      }
    }
  }
}

// ------------------------------------------------------------ fixed: tile
// Non-identity fixed layouts, every input read once as whole 16-byte chunks
// and every output written as whole 16-byte chunks (numerics: 56-byte
// native, 44-byte wire; the group kernel above reads each output chunk's
// terms as 8-byte windows, 32 bytes of loads per 16 written).  A workgroup
// takes tiles of kTileRec records: the tile's input chunks into LDS (the
// next tile's loads in flight meanwhile), one lane per record builds its
// output words from the term program -- the same for every lane, so it
// lives in scalar registers (kernel arguments) -- into an LDS output tile,
// and the tile leaves as 16-byte stores.  Records of up to IW input and OW
// output words, up to KT terms per output word.
constexpr uint32_t kTileRec = 256;
template <int OW, int KT>
struct tile_prog {
  uint32_t src[OW][KT];  // input word of the term (within the record)
  uint32_t sel[OW][KT];  // v_perm selector, or bool_term's with kGrpBool
  uint32_t nterm[OW];    // terms of the output word (0: a zero word)
};

template <int IW, int OW, int KT>
__global__ __launch_bounds__(256) void k_fixed_tile(const u32x4 *__restrict__ in, u32x4 *__restrict__ out,
                                                    uint64_t n, uint32_t in_w, uint32_t out_w,
                                                    const tile_prog<OW, KT> prog) {
  // LDS (dynamic): the input tile (+ 4 zero words), then the output tile
  extern __shared__ __attribute__((aligned(16))) uint32_t tsm[];
  uint32_t *tin = tsm, *tout = tsm + kTileRec * in_w + 4;
  constexpr int CH = (IW + 3) / 4;  // input chunks per lane per tile (at most)
  const uint32_t tid = threadIdx.x;
  const uint64_t ntiles = (n + kTileRec - 1) / kTileRec;
  if (tid < 4) tin[kTileRec * in_w + tid] = 0u;
  u32x4 v[CH];
  // input chunks of tile t into v (a partial chunk at the batch's end word
  // by word; the words past it read as 0)
  auto load = [&](uint64_t t) {
    const uint64_t nt = min<uint64_t>(kTileRec, n - t * kTileRec);
    const uint32_t nw = static_cast<uint32_t>(nt) * in_w, nc = (nw + 3u) >> 2;
    const u32x4 *src = in + t * kTileRec * in_w / 4u;  // (kTileRec * in_w words: whole chunks)
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const uint32_t c = tid + 256u * k;
      if (c + 1u < nc || (c + 1u == nc && !(nw & 3u))) {
        v[k] = src[c];
      } else if (c < nc) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(src + c);
        const uint32_t m = nw & 3u;
        v[k] = u32x4{w[0], m > 1 ? w[1] : 0u, m > 2 ? w[2] : 0u, 0u};
      }
    }
  };
  uint64_t t = blockIdx.x;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    const uint64_t nt = min<uint64_t>(kTileRec, n - t * kTileRec);
    const uint32_t nin = static_cast<uint32_t>(nt) * in_w;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const uint32_t c = tid + 256u * k;
      if (4u * c < nin) *reinterpret_cast<u32x4 *>(tin + 4u * c) = v[k];
    }
    __syncthreads();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);  // in flight during the build and the stores
    if (tid < nt) {
      const uint32_t *rin = tin + tid * in_w;
      uint32_t *rout = tout + tid * out_w;
#pragma unroll
      for (int j = 0; j < OW; ++j) {
        if (j < static_cast<int>(out_w)) {
          uint32_t o = 0;
#pragma unroll
          for (int k = 0; k < KT; ++k) {
            if (k < static_cast<int>(prog.nterm[j])) {
              const uint32_t a = prog.src[j][k], sl = prog.sel[j][k];
              if (sl & kGrpBool) o |= bool_term(rin[a], sl & 0xffffffu);
              else o |= perm(rin[a + 1], rin[a], sl);
            }
          }
          rout[j] = o;
        }
      }
    }
    __syncthreads();
    const uint32_t nout = static_cast<uint32_t>(nt) * out_w, noc = (nout + 3u) >> 2;
    u32x4 *dst = out + t * kTileRec * out_w / 4u;
    for (uint32_t c = tid; c < noc; c += 256u) {
      const u32x4 x = *reinterpret_cast<const u32x4 *>(tout + 4u * c);
      if (4u * c + 4u <= nout) {
        dst[c] = x;
      } else {
        uint32_t *w = reinterpret_cast<uint32_t *>(dst + c);
        const uint32_t m = nout & 3u;
        w[0] = x.x;
        if (m > 1) w[1] = x.y;
        if (m > 2) w[2] = x.z;
      }
    }
  }
}

}  // namespace dev
}  // namespace xdrg
