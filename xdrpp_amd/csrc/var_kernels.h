// Variable-length record kernels (opaque<>/string<>, unions, containers),
// written once over a *walker*: the per-record field walk of a plan.
//
//   var_encode_body<W>   one wave = 64 consecutive records (xdr_generic_put,
//                        xdrpp/marshal.h:84-137): offsets from the size
//                        pass's block base + a wave scan; the native tile in
//                        LDS; the lane-per-record walk writes scalar wire
//                        words into an LDS image of the wave's output stretch
//                        and registers its payloads; payloads are copied by
//                        a flat 16-byte chunk map (consecutive lanes,
//                        consecutive chunks); the image leaves with aligned
//                        16-byte stores.
//   var_decode_body<W>   one wave = 64 records (xdr_generic_get,
//                        marshal.h:142-211): the wave's input stretch read
//                        once into an LDS window and written once to the
//                        heap (the decoded heap is the stream itself); the
//                        lane-per-record walk parses from the window into an
//                        LDS native tile with every bound / pad /
//                        discriminant / enum check; the tile leaves with
//                        16-byte stores.
//   var_size_body<W>     xdr_size per record (xdrpp/types.h:240-244) + the
//                        64-record block sums the scan turns into offsets.
//
// Walkers: the plan interpreter (xdrgpu.hip, any plan) and the plan-
// specialized walkers that spec.cpp generates as straight-line code per
// plan and compiles with hiprtc.  A walker provides
//   bool enc(enc_ctx<K> &, const uint8_t *nat)
//   bool dec(dec_ctx<RA> &, uint8_t *nat)
//   uint64_t size(const uint8_t *nat, uint32_t &bad_op)
// and reports its own field errors through the context.
#pragma once
#include "dev_common.h"

namespace xdrg {
namespace dev {

// ---------------------------------------------------------------- encode
// LDS of an encode wave: the native tile is dead once the walk is done, so
// the chunk descriptors and the chunk map (built after the walk) reuse it;
// the image follows.  (Overlaying them cut recvar's LDS per wave from 16.4
// to 12.8 KiB: more waves per CU to hide the wave's memory round trips.)
struct enc_i_lds {
  uint32_t tile, desc, map, img, total;
};
__host__ __device__ inline enc_i_lds enc_i_layout(uint32_t stride, uint32_t KMAX, uint32_t MC,
                                                 uint32_t C) {
  enc_i_lds L;
  L.tile = 0;
  L.desc = 0;
  L.map = L.desc + 64u * KMAX * 16u;
  const uint32_t a = (64u * stride + 15u) & ~15u, b = L.map + ((MC * 2u + 15u) & ~15u);
  L.img = a > b ? a : b;
  L.total = L.img + C + 32u;  // phase shift + the last (partial) chunk read
  return L;
}

struct echunk_desc {  // 16 bytes: one payload slot of one lane
  uint64_t src;       // heap byte offset
  uint32_t dst;       // byte offset in the wave's stretch
  uint32_t len;       // payload bytes
};

// Store word `v` at stretch offset `at`: image if it fits, else global.
__device__ __forceinline__ void img_put(uint8_t *im, uint32_t C, uint8_t *gout, uint32_t at,
                                        uint32_t v) {
  if (at < C) *reinterpret_cast<uint32_t *>(im + at) = v;
  else st32(gout + at, v);
}

// One lane's encode state: where its next wire word goes (stretch offset
// `at`, stream offset `pos`), the checks of xdr_generic_put, and up to KMAX
// payload slots for the chunk map.  Payloads that do not take a slot (no
// slot left, longer than a chunk map entry can address, inside a container
// element) are copied by the lane itself.
template <int KMAX>
struct enc_ctx {
  uint8_t *im;
  uint32_t C;
  uint8_t *gout;
  const uint8_t *heap;
  uint64_t heap_len;
  uint64_t cap;
  uint32_t stack_limit;
  uint64_t r;
  unsigned long long *err;
  uint32_t at;
  uint64_t pos;
  uint64_t psr[KMAX];
  uint32_t pds[KMAX], pln[KMAX];

  // check(n) of xdr_generic_put (marshal.h:104-108) after the stack budget
  // of the field's class level (marshal.h:129-136)
  __device__ __forceinline__ bool field(uint32_t op, uint32_t depth, uint64_t need) {
    if (depth > stack_limit) {
      report(err, r, op, XDRG_ERR_STACK_PUT);
      return false;
    }
    if (need > cap - min(pos, cap)) {
      report(err, r, op, XDRG_ERR_OVERFLOW_PUT);
      return false;
    }
    return true;
  }
  __device__ __forceinline__ void put(uint32_t v) {
    img_put(im, C, gout, at, v);
    at += 4;
    pos += 4;
  }
  __device__ __forceinline__ void skip(uint32_t len) {
    const uint32_t p4 = (len + 3u) & ~3u;
    at += p4;
    pos += p4;
  }
  // payload of `len` bytes at heap offset `src`, copied by the chunk map
  template <int K> __device__ __forceinline__ void slot(uint64_t src, uint32_t len) {
    if (len) {
      psr[K] = src;
      pds[K] = at;
      pln[K] = len;
    }
    skip(len);
  }
  // the same, slot chosen at run time (interpreter walk)
  __device__ __forceinline__ void slot_dyn(uint32_t k, uint64_t src, uint32_t len) {
#pragma unroll
    for (int q = 0; q < KMAX; ++q)
      if (static_cast<uint32_t>(q) == k) { psr[q] = src; pds[q] = at; pln[q] = len; }
    skip(len);
  }
  // payload copied word by word by this lane (put_bytes, marshal.cc:59-72)
  __device__ void copy(uint64_t src, uint32_t len) {
    const uint32_t nw = (len + 3u) >> 2;
    for (uint32_t k = 0; k < nw; ++k) {
      uint32_t w = unaligned_word(heap, heap_len, src + 4ull * k);
      if (4u * k + 4u > len) w &= keep_mask(len - 4u * k);
      img_put(im, C, gout, at + 4u * k, w);
    }
    skip(len);
  }
  // a word of the heap (container elements), bytes past heap_len read 0
  __device__ __forceinline__ uint32_t hword(uint64_t off) const { return unaligned_word(heap, heap_len, off); }
};

template <class W, int KMAX, int U>
__device__ __forceinline__ void var_encode_body(
    const W &w, const uint8_t *__restrict__ native, uint64_t n, uint32_t stride,
    const uint8_t *__restrict__ heap, uint64_t heap_len, uint8_t *__restrict__ xdr, uint64_t cap,
    uint64_t *__restrict__ offsets, const uint32_t *__restrict__ sizes,
    const unsigned long long *__restrict__ block_base, uint32_t stack_limit, uint32_t MC,
    uint32_t C, uint32_t mark, unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  const enc_i_lds L = enc_i_layout(stride, KMAX, MC, C);
  uint8_t *tile = sm + L.tile;
  echunk_desc *desc = reinterpret_cast<echunk_desc *>(sm + L.desc);
  uint16_t *map = reinterpret_cast<uint16_t *>(sm + L.map);
  uint8_t *img = sm + L.img;
  const uint32_t lane = threadIdx.x;
  const uint64_t wr0 = static_cast<uint64_t>(blockIdx.x) * 64u;
  const uint64_t r = wr0 + lane;
  const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(64, n - wr0));

  // ---- record offsets: wave scan of the sizes on top of the block base
  // (sizes, block base and the native tile are loaded in one round trip)
  const uint32_t sz = r < n ? sizes[r] : kSizeErr;
  const uint64_t wave_out = block_base[blockIdx.x];
  stage_tile(tile, native + wr0 * stride, nrec * stride, lane, 64u);
  const bool szok = !(sz & kSizeErr);
  const unsigned long long v = szok ? sz : 0ull;
  unsigned long long incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long x = __shfl_up(incl, o, 64);
    if (lane >= static_cast<uint32_t>(o)) incl += x;
  }
  const uint64_t T = rl64(incl, 63);  // bytes of the wave's stretch
  const uint64_t off = wave_out + incl - v;
  if (r < n) offsets[r] = off;
  wave_sync();

  const uint32_t sh = static_cast<uint32_t>(wave_out & 15u);
  uint8_t *im = img + sh;          // image byte j <-> global wave_out + j
  uint8_t *gout = xdr + wave_out;  // direct path for j >= C

  // ---- walk: scalar words -> image, payload slots -> registers
  enc_ctx<KMAX> c;
  c.im = im;
  c.C = C;
  c.gout = gout;
  c.heap = heap;
  c.heap_len = heap_len;
  c.cap = cap;
  c.stack_limit = stack_limit;
  c.r = r;
  c.err = err;
  c.at = static_cast<uint32_t>(off - wave_out);
  c.pos = off;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) { c.psr[k] = 0; c.pds[k] = 0; c.pln[k] = 0; }
  bool ok = szok;
  if (ok && mark) {  // the message's record mark (message_t::alloc, marshal.cc:15-31)
    if (4 > cap - min(c.pos, cap)) {
      report(err, r, kOpRecordLevel, XDRG_ERR_OVERFLOW_PUT);
      ok = false;
    } else {
      c.put(mark_word(sz - 4u));
    }
  }
  ok = w.enc(c, tile + lane * stride, ok);
  if (!ok) {  // a failing record's bytes are unspecified (never past `cap`)
#pragma unroll
    for (int k = 0; k < KMAX; ++k) c.pln[k] = 0;
  }
  wave_sync();  // every lane's walk is done with the tile: the chunk map reuses it

  // ---- chunk map: u16 lane << 10 | slot << 8 | chunk
  uint32_t nch = 0;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) nch += (c.pln[k] + 15u) >> 4;
  uint32_t cincl = nch;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(cincl, o, 64);
    if (lane >= static_cast<uint32_t>(o)) cincl += x;
  }
  const uint32_t M = __shfl(cincl, 63, 64);
  {
    uint32_t e = cincl - nch;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (!c.pln[k]) continue;
      desc[lane * KMAX + k] = echunk_desc{c.psr[k], c.pds[k], c.pln[k]};
      const uint32_t nq = (c.pln[k] + 15u) >> 4;
      const uint32_t tag = (lane << 10) | (static_cast<uint32_t>(k) << 8);
      for (uint32_t q = 0; q < nq; ++q) map[e + q] = static_cast<uint16_t>(tag | q);
      e += nq;
    }
  }
  wave_sync();

  // ---- payload chunks: heap -> image, U chunks in flight per lane.  Three
  // passes per batch: the chunk descriptors (LDS), then the U loads with no
  // use of a loaded value in between (so none waits for another), then the
  // rare chunk that ends past the heap, the pad masks and the stores.
  for (uint32_t c0 = 0; c0 < M; c0 += 64u * U) {
    u32x4 val[U];
    uint64_t hs[U];
    uint32_t at[U], nb[U], rem[U];
    bool fast[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t ci = c0 + 64u * u + lane;
      nb[u] = 0u;
      at[u] = 0u;
      hs[u] = 0u;
      rem[u] = 16u;
      fast[u] = false;
      if (ci < M) {
        const uint32_t m = map[ci];
        const echunk_desc d = desc[(m >> 10) * KMAX + ((m >> 8) & 3u)];
        const uint32_t q16 = (m & 0xffu) << 4;
        hs[u] = d.src + q16;
        rem[u] = d.len - q16;
        at[u] = d.dst + q16;
        nb[u] = min(16u, ((d.len + 3u) & ~3u) - q16);
        fast[u] = hs[u] + 16u <= heap_len;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (fast[u]) val[u] = ld16u(heap + hs[u]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!nb[u]) continue;
      u32x4 x = val[u];
      if (!fast[u])
        x = u32x4{unaligned_word(heap, heap_len, hs[u]), unaligned_word(heap, heap_len, hs[u] + 4),
                  unaligned_word(heap, heap_len, hs[u] + 8), unaligned_word(heap, heap_len, hs[u] + 12)};
      const int32_t rm = static_cast<int32_t>(rem[u]);
      if (rm < 16) {  // zero the pad bytes after the payload (put_bytes)
        x.x &= keep_bytes(rm);
        x.y &= keep_bytes(rm - 4);
        x.z &= keep_bytes(rm - 8);
        x.w &= keep_bytes(rm - 12);
      }
      if (at[u] + 16u <= C) {
        uint32_t *wp = reinterpret_cast<uint32_t *>(im + at[u]);
        wp[0] = x.x;
        if (nb[u] > 4u) wp[1] = x.y;
        if (nb[u] > 8u) wp[2] = x.z;
        if (nb[u] > 12u) wp[3] = x.w;
      } else if (at[u] >= C && nb[u] == 16u) {
        st16u(gout + at[u], x);  // a whole chunk past the image: one (4-aligned) 16-byte store
      } else {
        img_put(im, C, gout, at[u], x.x);
        if (nb[u] > 4u) img_put(im, C, gout, at[u] + 4, x.y);
        if (nb[u] > 8u) img_put(im, C, gout, at[u] + 8, x.z);
        if (nb[u] > 12u) img_put(im, C, gout, at[u] + 12, x.w);
      }
    }
  }
  wave_sync();

  // ---- image -> global: aligned 16-byte chunks, partial words at the edges
  {
    const uint64_t gs = wave_out;
    const uint64_t ge = min<uint64_t>(gs + min<uint64_t>(T, C), cap);
    if (ge > gs) {
      const uint64_t c0 = gs & ~15ull;
      const uint32_t nc = static_cast<uint32_t>((ge - c0 + 15u) >> 4);
      for (uint32_t ci = lane; ci < nc; ci += 64u) {
        const uint64_t ca = c0 + 16ull * ci;
        const uint8_t *lsrc = img + 16u * ci;  // img + sh <-> gs, and gs - sh = c0
        if (ca >= gs && ca + 16u <= ge) {
          *reinterpret_cast<u32x4 *>(xdr + ca) = *reinterpret_cast<const u32x4 *>(lsrc);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint64_t wa = ca + 4u * q;
            if (wa >= gs && wa + 4u <= ge) st32(xdr + wa, *reinterpret_cast<const uint32_t *>(lsrc + 4 * q));
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- decode
__host__ __device__ inline uint32_t dec_w_lds(uint32_t stride, uint32_t C) {
  return ((64u * stride + 15u) & ~15u) + C + 32u;
}

// Stream reader of a wave: the window for stream bytes in [ws, ws + wc),
// global memory otherwise.  Past the window a lane keeps a 32-byte
// read-ahead of the stream (two aligned 16-byte chunks loaded together):
// consecutive fields are adjacent, so one round trip serves up to 8 words
// instead of 1.  The second chunk is loaded only when it holds stream bytes
// (an aligned chunk with a stream byte never leaves the stream's pages).
template <bool RA>
struct win_reader {
  const uint8_t *xdr;
  uint64_t len, ws, wc;
  const uint8_t *wnd;
  uint32_t sh;
  uintptr_t xbase, xend, ra_line;
  u32x4 ra0, ra1;
  __device__ __forceinline__ uint32_t operator()(uint64_t pos) {
    const uint64_t rel = pos - ws;
    if (pos >= ws && rel + 4 <= wc) {
      const uint8_t *q = wnd + rel;
      if (((sh + rel) & 3u) == 0) return *reinterpret_cast<const uint32_t *>(q);
      return uint32_t(q[0]) | (uint32_t(q[1]) << 8) | (uint32_t(q[2]) << 16) | (uint32_t(q[3]) << 24);
    }
    const uintptr_t ga = xbase + pos;
    if (!RA || (ga & 3u) || pos + 4 > len) return unaligned_word(xdr, len, pos);
    if (ga - ra_line >= 32u) {
      ra_line = ga & ~uintptr_t(15);
      ra0 = *reinterpret_cast<const u32x4 *>(ra_line);
      ra1 = ra_line + 16u < xend ? *reinterpret_cast<const u32x4 *>(ra_line + 16u) : u32x4{0u, 0u, 0u, 0u};
    }
    const uint32_t k = static_cast<uint32_t>(ga - ra_line) >> 2;
    const u32x4 h = k < 4u ? ra0 : ra1;
    const uint32_t j = k & 3u;
    return j == 0 ? h.x : j == 1 ? h.y : j == 2 ? h.z : h.w;
  }
};

// One lane's decode state: the stream position `p` inside its record
// [.., b), the checks of xdr_generic_get, and the bump pointer of the
// record's element arrays (xvector<T> / pointer<T>) in the decoded heap.
template <bool RA>
struct dec_ctx {
  win_reader<RA> rd;
  uint64_t p, b;
  uint32_t stack_limit;
  uint64_t r;
  unsigned long long *err;
  uint8_t *heap;  // decoded heap (element arrays live at ecur)
  uint64_t ecur;

  // stack budget, then check(n) of xdr_generic_get (marshal.h:166-170)
  __device__ __forceinline__ bool field(uint32_t op, uint32_t depth, uint64_t need) {
    if (depth > stack_limit) {
      report(err, r, op, XDRG_ERR_STACK_GET);
      return false;
    }
    if (b - p < need) {
      report(err, r, op, XDRG_ERR_OVERFLOW_GET);
      return false;
    }
    return true;
  }
  __device__ __forceinline__ uint32_t word() {  // raw (big-endian) wire word
    const uint32_t v = rd(p);
    p += 4;
    return v;
  }
  __device__ __forceinline__ uint32_t peek(uint64_t at) { return rd(at); }
  __device__ __forceinline__ bool fail(uint32_t op, uint32_t code) {
    report(err, r, op, code);
    return false;
  }
};

template <class W, bool COPY, bool RA>
__device__ __forceinline__ void var_decode_body(
    const W &w, const uint8_t *__restrict__ xdr, uint64_t len, const uint64_t *__restrict__ offsets,
    uint64_t n, uint8_t *__restrict__ native, uint32_t stride, uint8_t *__restrict__ heap,
    uint32_t stack_limit, uint32_t C, uint64_t ebase, uint32_t F, uint32_t mark,
    unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  const uint32_t lane = threadIdx.x;
  const uint32_t tile_bytes = (64u * stride + 15u) & ~15u;
  uint8_t *tile = sm;
  uint8_t *win = sm + tile_bytes;
  const uint64_t wr0 = static_cast<uint64_t>(blockIdx.x) * 64u;
  const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(64, n - wr0));
  const uint64_t r = wr0 + lane;
  uint64_t a = 0, b = 0;
  if (lane < nrec) {
    a = offsets[r];
    b = offsets[r + 1];
  }
  // the wave's stretch, clamped to the stream (bad indices are reported by
  // the per-record checks below; the window just gets smaller)
  const uint64_t ws = min<uint64_t>(rl64(a, 0), len);
  const uint64_t we = max<uint64_t>(ws, min<uint64_t>(rl64(b, nrec - 1), len));
  const uint64_t wc = min<uint64_t>(we - ws, C);  // bytes held in the window
  const uintptr_t gbase = reinterpret_cast<uintptr_t>(xdr) + ws;
  const uint32_t sh = static_cast<uint32_t>(gbase & 15u);

  for (uint32_t i = lane; i < tile_bytes / 16u; i += 64u)
    reinterpret_cast<u32x4 *>(tile)[i] = u32x4{0u, 0u, 0u, 0u};
  {
    // Aligned 16-byte chunks covering the stretch [ws, we), 8 loads in
    // flight per lane.  A chunk never leaves the pages that hold stream
    // bytes, so edge chunks load whole; only in-range words reach the heap.
    // Chunks inside [ws, ws + wc) also fill the window.
    const uint32_t nwin = static_cast<uint32_t>((sh + wc + 15u) >> 4);
    const uint64_t nall = COPY ? (sh + (we - ws) + 15u) >> 4 : nwin;
    const uint8_t *g0 = xdr + ws - sh;
    constexpr int UL = 8;
    for (uint64_t c0 = 0; c0 < nall; c0 += 64u * UL) {
      u32x4 v[UL];
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const uint64_t ci = c0 + 64u * u + lane;
        if (ci < nall) v[u] = *reinterpret_cast<const u32x4 *>(g0 + 16u * ci);
      }
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const uint64_t ci = c0 + 64u * u + lane;
        if (ci >= nall) continue;
        if (ci < nwin) reinterpret_cast<u32x4 *>(win)[ci] = v[u];
        if (COPY) {
          const int64_t o = static_cast<int64_t>(16u * ci) - sh;  // stream offset - ws
          const int64_t lim = static_cast<int64_t>(we - ws);
          uint8_t *hd = heap + ws + o;
          if (o >= 0 && o + 16 <= lim) {
            st16u(hd, v[u]);
          } else {
            const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (o + 4 * q >= 0 && o + 4 * q + 4 <= lim) st32(hd + 4 * q, w4[q]);
          }
        }
      }
    }
  }
  wave_sync();

  dec_ctx<RA> c;
  c.rd.xdr = xdr;
  c.rd.len = len;
  c.rd.ws = ws;
  c.rd.wc = wc;
  c.rd.wnd = win + sh;  // window byte j <-> stream byte ws + j
  c.rd.sh = sh;
  c.rd.xbase = reinterpret_cast<uintptr_t>(xdr);
  c.rd.xend = c.rd.xbase + len;
  c.rd.ra_line = ~uintptr_t(0);
  c.rd.ra0 = u32x4{0u, 0u, 0u, 0u};
  c.rd.ra1 = c.rd.ra0;
  c.p = a + mark;
  c.b = b;
  c.stack_limit = stack_limit;
  c.r = r;
  c.err = err;
  c.heap = heap;
  c.ecur = ebase + static_cast<uint64_t>(F) * a;  // this record's element arrays
  {
    uint8_t *nat = tile + lane * stride;
    bool ok = false;
    if (lane < nrec) {
      // xdr_from_msg: the message read_message framed (srpc.cc:29-55)
      const uint32_t mc = !mark || b < a || b > len ? 0u
                          : b - a < 4 ? XDRG_ERR_MSG_EOF : mark_code(c.rd(a), b - a - 4);
      if (r == n - 1 && b != len) report(err, n, kOpRecordLevel, XDRG_ERR_TRAILING);
      if (b < a || b > len) report(err, r, 0, XDRG_ERR_OVERFLOW_GET);
      else if (mc) report(err, r, kOpRecordLevel, mc);
      else if ((b - a) & 3u) report(err, r, kOpRecordLevel, XDRG_ERR_SIZE_NOT_MULT4);
      else ok = true;
    }
    ok = w.dec(c, nat, ok);
    if (ok && c.p != b) report(err, r, kOpRecordLevel, XDRG_ERR_TRAILING);
  }
  wave_sync();
  uint8_t *ndst = native + wr0 * stride;
  const uint32_t nbytes = nrec * stride;
  for (uint32_t i = lane; i < nbytes / 16u; i += 64u)
    reinterpret_cast<u32x4 *>(ndst)[i] = reinterpret_cast<const u32x4 *>(tile)[i];
  for (uint32_t i = (nbytes / 16u) * 4u + lane; i < nbytes / 4u; i += 64u)
    reinterpret_cast<uint32_t *>(ndst)[i] = reinterpret_cast<const uint32_t *>(tile)[i];
}

// ------------------------------------------------------------------ size
// One 64-thread workgroup = 64 consecutive records, natives staged in LDS
// with coalesced 16-byte loads.  sizes[r] = xdr_size (kSizeErr on a bad
// discriminant, reported as the size pass of k_var_size does), block_sums
// = the 64-record sums.
template <class W>
__device__ __forceinline__ void var_size_body(const W &w, const uint8_t *__restrict__ native, uint64_t n,
                                              uint32_t stride, uint32_t *__restrict__ sizes,
                                              unsigned long long *__restrict__ block_sums,
                                              uint32_t mark, unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
  const uint32_t lane = threadIdx.x;
  const uint64_t wr0 = static_cast<uint64_t>(blockIdx.x) * 64u;
  const uint64_t r = wr0 + lane;
  const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(64, n - wr0));
  const uint8_t *nsrc = native + wr0 * stride;
  if ((reinterpret_cast<uintptr_t>(nsrc) & 15u) == 0) {
    stage_tile(tile, nsrc, nrec * stride, lane, 64u);
  } else {
    for (uint32_t i = lane; i < nrec * stride / 4u; i += 64u)
      reinterpret_cast<uint32_t *>(tile)[i] = reinterpret_cast<const uint32_t *>(nsrc)[i];
  }
  wave_sync();
  uint32_t size = 0;
  if (r < n) {
    uint32_t bad_op = 0xffffffffu;
    const uint64_t s = w.size(tile + lane * stride, bad_op) + mark;
    if (bad_op != 0xffffffffu) {
      report(err, r, bad_op, XDRG_ERR_BAD_DISCRIMINANT);
      size = kSizeErr;
    } else if (s >= kSizeErr) {
      report(err, r, 0, XDRG_ERR_OVERFLOW_PUT);
      size = kSizeErr;
    } else {
      size = static_cast<uint32_t>(s);
    }
    if (sizes) sizes[r] = size;
  }
  unsigned long long v = (size & kSizeErr) ? 0ull : size;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (block_sums && lane == 0) block_sums[blockIdx.x] = v;
}

}  // namespace dev
}  // namespace xdrg
