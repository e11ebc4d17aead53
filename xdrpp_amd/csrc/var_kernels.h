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
//   bool enc(CTX &, const uint8_t *nat)  (CTX: an enc_ctx, checked or not)
//   bool dec(dec_ctx<RA> &, uint8_t *nat)
//   uint64_t size(const uint8_t *nat, const uint8_t *heap, uint64_t heap_len, uint32_t &bad_op)
// and reports its own field errors through the context.
#pragma once
#include "dev_common.h"

// Phase timestamps of a wave for tuning harnesses (tools/tune/enc_stamps.py
// defines XDRG_STAMP(k) before including the kernels); nothing in the
// library.
#ifndef XDRG_STAMP
#define XDRG_STAMP(k) ((void)0)
#endif
#ifndef XDRG_DSTAMP
#define XDRG_DSTAMP(k) ((void)0)
#endif
#ifndef XDRG_STAMPV
#define XDRG_STAMPV(k, v) ((void)0)
#endif
// Memory hints of the encode (tools/tune/enc_stamps.py CFLAGS A/B,
// profiles/r02s/nt_hints/): bit 0 non-temporal payload loads, bit 1
// non-temporal stream stores.  Stores: encode kernel -7 % recvar, -3 % rpc
// alone; enc+dec bench lines +0-2 %.
#ifndef XDRG_ENC_NT
#define XDRG_ENC_NT 2
#endif
// Waves per SIMD the walk-first record kernels are compiled for
// (__launch_bounds__'s second argument; tools/tune/stream_stamps.py
// CFLAGS=-DXDRG_PRE_WAVES=n, profiles/r04ad): 5 caps them at 96 VGPRs --
// recvar even (0.080 vs 0.081 ms), rpc spills (0.141 vs 0.117); 6: 0.12 /
// 0.20 ms.  4 is what they need anyway (102-105 VGPRs).
#ifndef XDRG_PRE_WAVES
#define XDRG_PRE_WAVES 4
#endif
// Non-temporal stores of the decode's heap copy (A/B, profiles/r02s/
// nt_hints/dnt*.log: recvar 0.089 -> 0.084 ms, vecrec 0.153 -> 0.137, rpc
// 0.120 -> 0.121).
#ifndef XDRG_DEC_NT
#define XDRG_DEC_NT 1
#endif
// Encode window pipelining (A/B: tools/tune/enc_stamps.py CFLAGS
// -DXDRG_ENC_PIPE=0/1): the next window's first payload batch is loaded
// before the current window's stores are issued, and the stores of a full
// window are a fixed number of buffer stores per lane (out-of-range lanes
// dropped by the descriptor's range check), so that waiting on those loads
// does not wait on the stores too (gfx9: loads and stores share vmcnt).
// The loads are inline asm the compiler does not count, waited for by an
// explicit vmcnt(SW) after the SW stores (tools/gpu/isa_audit.py checks the
// shape in the compiled code).  MI355X, 1M records, kernel alone
// (profiles/r03f): rpc 0.1616 -> 0.1582 ms, vecrec 0.0977 -> 0.0969,
// recvar 0.1073 -> 0.1066.
#ifndef XDRG_ENC_PIPE
#define XDRG_ENC_PIPE 1
#endif

namespace xdrg {
namespace dev {

// ---------------------------------------------------------------- encode
template <bool B> struct bool_tag { static constexpr bool value = B; };

// The 16 bytes at heap offset hs, bytes at or past len reading 0, for a
// chunk within 16 bytes of the heap's end (hs + 16 > len).  One 16-byte
// load ending at the heap's end and a byte shift; a heap shorter than 16
// bytes is read byte by byte, each load waited for inside its own asm
// statement so that no load of this rare path stays pending in the
// compiler's count (the pipelined windows count their own loads).
__device__ __forceinline__ u32x4 heap_tail16(const uint8_t *heap, uint64_t len, uint64_t hs) {
  if (hs >= len) return u32x4{0u, 0u, 0u, 0u};
  if (len >= 16) {
    const u32x4 t = ld16u(heap + len - 16);
    const uint32_t d = static_cast<uint32_t>(hs - (len - 16));  // 1..15: bytes of t before hs
    const uint32_t w = d >> 2, sb = d & 3u;
    const uint32_t t0 = w == 0 ? t.x : w == 1 ? t.y : w == 2 ? t.z : t.w;
    const uint32_t t1 = w == 0 ? t.y : w == 1 ? t.z : w == 2 ? t.w : 0u;
    const uint32_t t2 = w == 0 ? t.z : w == 1 ? t.w : 0u;
    const uint32_t t3 = w == 0 ? t.w : 0u;
    return u32x4{__builtin_amdgcn_alignbyte(t1, t0, sb), __builtin_amdgcn_alignbyte(t2, t1, sb),
                 __builtin_amdgcn_alignbyte(t3, t2, sb), __builtin_amdgcn_alignbyte(0u, t3, sb)};
  }
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  for (uint32_t k = 0; k < 16u && hs + k < len; ++k) {
    uint32_t byte;
    asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(byte) : "v"(heap + hs + k) : "memory");
    v[k >> 2] |= byte << (8u * (k & 3u));
  }
  return u32x4{v[0], v[1], v[2], v[3]};
}

// s_waitcnt vmcnt(N) that also defines `v` (loaded by inline asm the
// compiler does not count): nothing reads v before this wait.  The loads
// and the wait carry "; xb1" (tools/isa_audit.py pairs them in the
// compiled code).
template <uint32_t N, int U>
__device__ __forceinline__ void vm_wait_after(u32x4 (&v)[U]) {
  if constexpr (U == 2)
    asm volatile("s_waitcnt vmcnt(%2) ; xb1" : "+v"(v[0]), "+v"(v[1]) : "n"(N) : "memory");
  else if constexpr (U == 4)
    asm volatile("s_waitcnt vmcnt(%4) ; xb1" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) : "n"(N) : "memory");
  else if constexpr (U == 8)
    asm volatile("s_waitcnt vmcnt(%8) ; xb1"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                 : "n"(N) : "memory");
}

// LDS of an encode wave: the native tile (kept for every window round), the
// payload slots of the 64 lanes, their inclusive chunk counts, and the image
// of one window of the wave's output stretch.
struct enc_lds {
  uint32_t tile, desc, cum, img, total;
};
__host__ __device__ inline enc_lds enc_layout(uint32_t stride, uint32_t KMAX, uint32_t C) {
  enc_lds L;
  L.tile = 0;
  L.desc = (64u * stride + 15u) & ~15u;
  L.cum = L.desc + 64u * KMAX * 16u;
  L.img = L.cum + 64u * 4u;
  L.total = L.img + C + 32u;  // + the last (partial) chunk read
  return L;
}

struct echunk_desc {  // 16 bytes: one payload slot of one lane
  uint64_t src;       // heap byte offset
  uint32_t dst;       // image-space byte offset of the payload (below)
  uint32_t len;       // payload bytes
};

// One lane's encode state.  Positions are *image-space* offsets: stretch
// offset + the wave's 16-byte phase, so that window w = [w0, w0 + C) of
// image space maps onto whole aligned 16-byte chunks of the stream.  The
// walk stores only the words of the current window (LDS image); payloads
// in registered slots are copied by the wave's chunk pass; the rest
// (container elements, payloads past the slots) word by word by the lane.
// WL > 0 (word-list walk, plans whose scalar words per record are bounded
// by WL and whose payloads all take slots): the walk runs once and puts the
// record's scalar words in a list (LDS, word-major: word j of the lane at
// sw[64 j]); `rb[k]` = words before slot k.  Each window then places the
// list's words that land in it (emit_words) instead of walking again.
template <int KMAX, bool CHECK = true, int WL = 0>
struct enc_ctx {
  uint8_t *img;
  uint32_t w0, C;
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
  uint32_t *sw;  // WL: this lane's column of the word list
  uint32_t nw;   // WL: words listed
  uint32_t rb[KMAX > 0 ? KMAX : 1];

  // word `v` at image-space offset `a`, if it lies in the window
  __device__ __forceinline__ void wput(uint32_t a, uint32_t v) {
    if (a - w0 < C) *reinterpret_cast<uint32_t *>(img + (a - w0)) = v;
  }
  // check(n) of xdr_generic_put (marshal.h:104-108) after the stack budget
  // of the field's class level (marshal.h:129-136)
  __device__ __forceinline__ bool field(uint32_t op, uint32_t depth, uint64_t need) {
    if constexpr (!CHECK) return true;  // the wave fits `cap` and the plan's depth fits the budget
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
    if constexpr (WL > 0) {
      sw[64u * nw] = v;
      ++nw;
    } else {
      wput(at, v);
    }
    at += 4;
    pos += 4;
  }
  __device__ __forceinline__ void skip(uint32_t len) {
    const uint32_t p4 = (len + 3u) & ~3u;
    at += p4;
    pos += p4;
  }
  // payload of `len` bytes at heap offset `src`, copied by the chunk pass
  template <int K> __device__ __forceinline__ void slot(uint64_t src, uint32_t len) {
    if (len) {
      psr[K] = src;
      pds[K] = at;
      pln[K] = len;
    }
    if constexpr (WL > 0) rb[K] = nw;
    skip(len);
  }
  // the same, slot chosen at run time (interpreter walk)
  __device__ __forceinline__ void slot_dyn(uint32_t k, uint64_t src, uint32_t len) {
#pragma unroll
    for (int q = 0; q < KMAX; ++q)
      if (static_cast<uint32_t>(q) == k) { psr[q] = src; pds[q] = at; pln[q] = len; }
    skip(len);
  }
  // payload copied word by word by this lane (put_bytes, marshal.cc:59-72):
  // only the words of the window are read
  __device__ void copy(uint64_t src, uint32_t len) {
    const uint32_t nw = (len + 3u) >> 2;
    const uint32_t k0 = w0 > at ? (w0 - at) >> 2 : 0u;
    const uint32_t k1 = min(nw, w0 + C > at ? (w0 + C - at + 3u) >> 2 : 0u);
    for (uint32_t k = k0; k < k1; ++k) {
      uint32_t w = unaligned_word(heap, heap_len, src + 4ull * k);
      if (4u * k + 4u > len) w &= keep_mask(len - 4u * k);
      wput(at + 4u * k, w);
    }
    skip(len);
  }
  // a word of the heap (container elements), bytes past heap_len read 0
  __device__ __forceinline__ uint32_t hword(uint64_t off) const { return unaligned_word(heap, heap_len, off); }

  // the same state under the other checking mode, and back
  template <bool B>
  __device__ __forceinline__ enc_ctx<KMAX, B, WL> as() const {
    enc_ctx<KMAX, B, WL> o;
    o.img = img; o.w0 = w0; o.C = C; o.heap = heap; o.heap_len = heap_len; o.cap = cap;
    o.stack_limit = stack_limit; o.r = r; o.err = err; o.at = at; o.pos = pos;
    o.sw = sw; o.nw = nw;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) { o.psr[k] = psr[k]; o.pds[k] = pds[k]; o.pln[k] = pln[k]; o.rb[k] = rb[k]; }
    return o;
  }
  template <bool B>
  __device__ __forceinline__ void take(const enc_ctx<KMAX, B, WL> &o) {
    at = o.at;
    pos = o.pos;
    nw = o.nw;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) { psr[k] = o.psr[k]; pds[k] = o.pds[k]; pln[k] = o.pln[k]; rb[k] = o.rb[k]; }
  }
};

// Direct mode of an encode wave whose stretch could pass 2 GiB (some
// record of 32 MiB or more; unbounded plans): the lane writes its record
// straight to the stream, words and payloads alike, at 64-bit positions --
// xdr_generic_put record by record, with no window.
struct enc_direct_ctx {
  uint8_t *xdr;
  const uint8_t *heap;
  uint64_t heap_len;
  uint64_t cap;
  uint32_t stack_limit;
  uint64_t r;
  unsigned long long *err;
  uint64_t pos;

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
    st32(xdr + pos, v);
    pos += 4;
  }
  __device__ void copy(uint64_t src, uint32_t len) {  // put_bytes (marshal.cc:59-72), pad zeroed
    const uint32_t nw = (len + 3u) >> 2;
    for (uint32_t k = 0; k < nw; ++k) {
      uint32_t w = unaligned_word(heap, heap_len, src + 4ull * k);
      if (4u * k + 4u > len) w &= keep_mask(len - 4u * k);
      st32(xdr + pos + 4ull * k, w);
    }
    pos += 4ull * nw;
  }
  template <int K> __device__ __forceinline__ void slot(uint64_t src, uint32_t len) { copy(src, len); }
  __device__ __forceinline__ uint32_t hword(uint64_t off) const { return unaligned_word(heap, heap_len, off); }
};

// Word-list walk: the listed words of a lane's record (first byte at
// image-space offset a0) that land in the window [w0, w0 + C) -> image.
// Word j sits after the padded payloads of the slots listed before it.
template <int KMAX, bool B, int WL>
__device__ __forceinline__ void emit_words(const enc_ctx<KMAX, B, WL> &c, uint32_t a0) {
  uint32_t v[WL];
#pragma unroll
  for (int j = 0; j < WL; ++j)
    if (static_cast<uint32_t>(j) < c.nw) v[j] = c.sw[64u * j];
#pragma unroll
  for (int j = 0; j < WL; ++j) {
    uint32_t a = a0 + 4u * j;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (static_cast<uint32_t>(j) >= c.rb[k]) a += (c.pln[k] + 3u) & ~3u;
    if (static_cast<uint32_t>(j) < c.nw && a - c.w0 < c.C) *reinterpret_cast<uint32_t *>(c.img + (a - c.w0)) = v[j];
  }
}

// Chunks of a lane's slots that end at or before image-space offset `a`,
// and that start before `a` (the slots' chunks are in stream order).
template <int KMAX, bool B, int WL>
__device__ __forceinline__ uint32_t chunks_ending_by(const enc_ctx<KMAX, B, WL> &c, uint32_t a) {
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (c.pln[k] && a >= c.pds[k] + 16u) s += min((c.pln[k] + 15u) >> 4, (a - c.pds[k]) >> 4);
  return s;
}
template <int KMAX, bool B, int WL>
__device__ __forceinline__ uint32_t chunks_starting_before(const enc_ctx<KMAX, B, WL> &c, uint32_t a) {
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (c.pln[k] && a > c.pds[k]) s += min((c.pln[k] + 15u) >> 4, (a - c.pds[k] + 15u) >> 4);
  return s;
}

// ------------------------------------------------- decoupled look-back
constexpr unsigned long long kLbAgg = 1ull << 62;     // block total published
constexpr unsigned long long kLbIncl = 2ull << 62;    // block total + everything before it
constexpr unsigned long long kLbVal = (1ull << 62) - 1;
constexpr uint32_t kLbSpinLimit = 1u << 16;           // polls before a look-back gives up


typedef __attribute__((address_space(1))) unsigned long long lb_u64;
typedef __attribute__((address_space(1))) unsigned int lb_u32;
// generic -> global address space (agent-scope atomics on global, never flat)
__device__ __forceinline__ lb_u64 *lb_global(unsigned long long *p) { return (lb_u64 *)p; }

// Sum over the lanes of a wave (every lane active).
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
  for (int o = 32; o > 0; o >>= 1) x = min(x, static_cast<uint64_t>(__shfl_xor(x, o, 64)));
  return x;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t x) {
  for (int o = 32; o > 0; o >>= 1) x = max(x, static_cast<uint64_t>(__shfl_xor(x, o, 64)));
  return x;
}

// Decoupled look-back (single-pass chained scan): the exclusive prefix of
// block `blk`'s total.  desc[i] = state | value, one 8-byte word written by
// one store (the data is the flag).  Lane l reads blocks top - l - 64u,
// u < PER (64 PER blocks per poll: a poll is a round trip past the per-XCD
// L2s, so the window spans the waves resident at once -- 4 per lane took 4.3
// polls on average, profiles/r04s).  Returns false when a predecessor never
// published (kLbSpinLimit polls).
#ifndef XDRG_LB_PER
#define XDRG_LB_PER 16  // look-back window per poll, blocks per lane (tools/tune/stream_stamps.py CFLAGS)
#endif
template <int PER = XDRG_LB_PER>
__device__ __forceinline__ bool lookback(lb_u64 *desc, uint32_t blk, uint64_t &excl, uint32_t &polls) {
  constexpr uint32_t WIN = 64u * PER;
  const uint32_t lane = __lane_id();
  excl = 0;
  polls = 0;
  int64_t top = static_cast<int64_t>(blk) - 1;
  for (uint32_t spins = 0; top >= 0;) {
    uint64_t d[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t i = top - lane - 64 * u;
      d[u] = i >= 0 ? __hip_atomic_load(desc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbIncl;
    }
    ++polls;
    // first block (in look-back order) that has not published, and the
    // first that holds an inclusive prefix
    uint32_t dn = WIN, dp = WIN;
#pragma unroll
    for (int u = PER - 1; u >= 0; --u) {
      const unsigned long long mn = __ballot((d[u] >> 62) == 0u);
      const unsigned long long mp = __ballot((d[u] >> 62) == 2u);
      if (mn) dn = 64u * u + __builtin_ctzll(mn);
      if (mp) dp = 64u * u + __builtin_ctzll(mp);
    }
    const bool found = dp < dn;
    const uint32_t lim = found ? dp : dn;  // block totals (aggregates) summed by this step
    // the aggregates (each < 2^31: the launch guard 64 * max_rec < 2^31) in
    // two 16-bit-split parts, summed with DPP (no LDS) in u32: a part is at
    // most 64 * PER * 2^16 <= 2^28 over the wave
    static_assert(PER <= 64, "16-bit split sums must fit u32 over 64 * PER blocks");
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u)
      if (lane + 64u * u < lim) {
        lo += static_cast<uint32_t>(d[u]) & 0xffffu;
        hi += static_cast<uint32_t>((d[u] & kLbVal) >> 16);
      }
    excl += static_cast<uint64_t>(rl32(wave_incl_scan(lo), 63)) + (static_cast<uint64_t>(rl32(wave_incl_scan(hi), 63)) << 16);
    if (found) {  // + the inclusive prefix at dp
      uint64_t pv = 0;
#pragma unroll
      for (int u = 0; u < PER; ++u)
        if (dp / 64u == static_cast<uint32_t>(u)) pv = rl64(d[u], dp % 64u);
      excl += pv & kLbVal;
      return true;
    }
    top -= lim;
    if (dn < WIN) {  // a block before this one is still walking its records
      if (++spins > kLbSpinLimit) return false;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return true;
}

// One wave = 64 consecutive records (xdr_generic_put, marshal.h:84-137).
// The output stretch of the wave is produced in windows of C bytes of LDS
// image: per window the lanes whose record reaches into it walk it (scalar
// words of the window into the image), the wave copies the payload chunks
// that land in it (16-byte loads, consecutive lanes on consecutive chunks),
// and the window leaves as aligned, whole-line 16-byte stores.  No partial
// or scattered global store, so each 64-byte line of the stream is one
// write request to L2.
// NW > 0 (plan-specialized walks, whose field offsets are constants): the
// lane's record (NW words) is copied from the tile into registers before
// the walk, so the walk issues no LDS read -- its reads no longer wait
// behind its own image writes.  NW = 0: the walk reads the tile.
// WL (plans with a bounded scalar word list, W::kWords > 0, walked from
// registers): the list aliases the tile, which the walk no longer reads once
// the lane's record is in registers; the walk runs once, in the first round.
//
// PRE (word-list plans walked from registers without checks: the plan's
// depth fits the stack budget) -- no size pass: the walk runs first, with
// record-relative positions, and its byte counts are the sizes.
//   PRE = 1  the wave's base by a decoupled look-back over the byte totals of
//            the waves before it (xdrg_encode: no size pass, no scan);
//   PRE = 2  the base from block_base (xdrg_encode_sized after
//            xdrg_encode_sizes), the sizes not read.
// A wave whose bytes pass `cap` walks again with the checks to report the
// failing record (xdr_generic_put::check, marshal.h:104-108).
template <class W, int KMAX, int U, int NW = 0, uint32_t CMAX = 0, int PRE = 0>
__device__ __forceinline__ void var_encode_body(
    const W &w, const uint8_t *__restrict__ native, uint64_t n, uint32_t stride,
    const uint8_t *__restrict__ heap, uint64_t heap_len, uint8_t *__restrict__ xdr, uint64_t cap,
    uint64_t *__restrict__ offsets, const uint32_t *__restrict__ sizes,
    const unsigned long long *__restrict__ block_base, uint32_t stack_limit, uint32_t C,
    uint32_t mark, unsigned long long *err, unsigned long long *lbd = nullptr, uint32_t nb = 0,
    uint64_t *total = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  constexpr int WL = (W::kWords > 0 && NW > 0) ? static_cast<int>(W::kWords) + 1 : 0;  // + the mark
  // PRE, and register walks without a word list: no native tile -- the
  // lane loads its record straight into registers, and the tile's room
  // holds only the word list (rpc: 2.8 of 5 KiB), or nothing (vecrec,
  // containertest): more waves per CU
  constexpr bool RREG = NW > 0 && (PRE != 0 || WL == 0);
  const enc_lds L = enc_layout(PRE != 0 ? 4u * WL : RREG ? 0u : stride, KMAX, C);
  uint8_t *tile = sm + L.tile;
  echunk_desc *desc = reinterpret_cast<echunk_desc *>(sm + L.desc);
  uint32_t *cum = reinterpret_cast<uint32_t *>(sm + L.cum);
  uint8_t *img = sm + L.img;
  const uint32_t lane = threadIdx.x;
  const uint64_t wr0 = static_cast<uint64_t>(blockIdx.x) * 64u;
  const uint64_t r = wr0 + lane;
  const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(64, n - wr0));
  XDRG_STAMP(0);
  static_assert(PRE == 0 || (WL > 0 && W::kFastWalk), "the pre-walk runs on word-list plans");

  uint32_t sz, v, T;
  bool szok;
  uint64_t wave_out, off;
  enc_ctx<KMAX, true, WL> c;
  c.sw = reinterpret_cast<uint32_t *>(tile) + lane;
  c.nw = 0;
  c.img = img;
  c.C = C;
  c.heap = heap;
  c.heap_len = heap_len;
  c.cap = cap;
  c.stack_limit = stack_limit;
  c.r = r;
  c.err = err;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) { c.psr[k] = 0; c.pds[k] = 0; c.pln[k] = 0; c.rb[k] = 0; }
  uint32_t rec[NW > 0 ? NW : 1];
  // the record (16- or 8-byte loads: the host passes 16-aligned natives)
  auto load_rec = [&]() {
    const uint8_t *src = native + r * static_cast<uint64_t>(4 * (NW > 0 ? NW : 1));
#pragma unroll
    for (int k = 0; k < (NW > 0 ? NW : 1); ++k) rec[k] = 0u;
    if (lane < nrec) {
      if constexpr (NW % 4 == 0) {
#pragma unroll
        for (int k = 0; k < NW; k += 4) {
          const u32x4 q = *reinterpret_cast<const u32x4 *>(src + 4 * k);
          rec[k] = q.x; rec[k + 1] = q.y; rec[k + 2] = q.z; rec[k + 3] = q.w;
        }
      } else if constexpr (NW % 2 == 0) {
#pragma unroll
        for (int k = 0; k < NW; k += 2) {
          const uint2 q = *reinterpret_cast<const uint2 *>(src + 4 * k);
          rec[k] = q.x; rec[k + 1] = q.y;
        }
      } else {
#pragma unroll
        for (int k = 0; k < NW; ++k) rec[k] = ld32(src + 4 * k);
      }
    }
  };
  if constexpr (PRE != 0) {
    // ---- the walk first: the record's words into the list (tile), its
    // payloads into slots, its byte count
    if constexpr (PRE == 2) wave_out = block_base[blockIdx.x];
    load_rec();
    enc_ctx<KMAX, false, WL> f = c.template as<false>();
    f.at = 0;
    f.pos = 0;
    bool okw = r < n;
    if (okw && mark) f.put(0u);  // the record mark, set below
    okw = w.enc(f, reinterpret_cast<const uint8_t *>(rec), okw);
    if (r < n && !okw) {  // an unchecked walk fails only at a bad discriminant (gen_hh.cc:645,658)
      uint32_t bad = 0xffffffffu;
      (void)w.size(reinterpret_cast<const uint8_t *>(rec), heap, heap_len, bad);
      report(err, r, bad == 0xffffffffu ? 0u : bad, XDRG_ERR_BAD_DISCRIMINANT);
    }
    v = okw ? f.at : 0u;
    if (okw && mark) f.sw[0] = mark_word(v - 4u);
    szok = okw;
    sz = okw ? v : kSizeErr;
    if (!okw) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k) f.pln[k] = 0;
    }
    c.take(f);
    const uint32_t incl = wave_incl_scan(v);
    T = rl32(incl, 63);
    if constexpr (PRE == 1) {
      const uint32_t blk = blockIdx.x;
      if (lane == 0)
        __hip_atomic_store(lb_global(lbd) + blk, (blk == 0 ? kLbIncl : kLbAgg) | T, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      uint64_t excl = 0;
      uint32_t polls = 0;
      if (!lookback(lb_global(lbd), blk, excl, polls)) {
        report(err, wr0, kOpRecordLevel, XDRG_ERR_LOOKBACK);
        return;
      }
      XDRG_STAMPV(6, polls);
      if (blk > 0 && lane == 0)
        __hip_atomic_store(lb_global(lbd) + blk, kLbIncl | ((excl + T) & kLbVal), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      wave_out = excl;
      if (r + 1 == n) {  // offsets[n] and the total (k_scan_blocks' job in two passes)
        offsets[n] = wave_out + T;
        *total = wave_out + T;
      }
    }
    off = wave_out + (incl - v);
    if (r < n) offsets[r] = off;
    const uint32_t a0r = static_cast<uint32_t>(incl - v) + static_cast<uint32_t>(wave_out & 15u);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) c.pds[k] += a0r;  // image space
    // a wave whose bytes pass `cap`: the checks, in the reference's order;
    // the re-walk's list goes to the image (unused until the windows)
    if (wave_out + T > cap && r < n && okw) {
      enc_ctx<KMAX, true, WL> k = c;
      k.sw = reinterpret_cast<uint32_t *>(img) + lane;
      k.nw = 0;
      k.at = 0;
      k.pos = off;
#pragma unroll
      for (int q = 0; q < KMAX; ++q) { k.psr[q] = 0; k.pds[q] = 0; k.pln[q] = 0; k.rb[q] = 0; }
      bool okc = true;
      if (mark) {
        if (4 > cap - min(k.pos, cap)) {
          report(err, r, kOpRecordLevel, XDRG_ERR_OVERFLOW_PUT);
          okc = false;
        } else {
          k.put(mark_word(v - 4u));
        }
      }
      (void)w.enc(k, reinterpret_cast<const uint8_t *>(rec), okc);
    }
    wave_sync();
  } else {
  // ---- record offsets: wave scan of the sizes on top of the block base
  // (sizes, block base and the native tile are loaded in one round trip)
  sz = r < n ? sizes[r] : kSizeErr;
  wave_out = block_base[blockIdx.x];
  if constexpr (RREG) load_rec();
  else stage_tile<8>(tile, native + wr0 * stride, nrec * stride, lane, 64u);
  szok = !(sz & kSizeErr);
  v = szok ? sz : 0u;
  if constexpr (W::kDirect) {
    if (__any(v >= (1u << 25))) {  // 64 records could pass 2^31 bytes: direct mode
      uint64_t inc = v;
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t x = __shfl_up(inc, o, 64);
        if (lane >= static_cast<uint32_t>(o)) inc += x;
      }
      const uint64_t doff = wave_out + inc - v;
      if (r < n) offsets[r] = doff;
      wave_sync();  // the tile
      if (r >= n || !szok) return;
      enc_direct_ctx d{xdr, heap, heap_len, cap, stack_limit, r, err, doff};
      if (mark) {  // the message's record mark (message_t::alloc, marshal.cc:15-31)
        if (!d.field(kOpRecordLevel, 0, 4)) return;
        d.put(mark_word(sz - 4u));
      }
      if constexpr (RREG) (void)w.enc(d, reinterpret_cast<const uint8_t *>(rec), true);
      else (void)w.enc(d, tile + lane * stride, true);
      return;
    }
  }
  const uint32_t incl = wave_incl_scan(v);  // a wave's stretch < 2^31 bytes (direct mode above)
  T = rl32(incl, 63);                       // bytes of the wave's stretch
  off = wave_out + (incl - v);
  if (r < n) offsets[r] = off;
  wave_sync();
  }
  XDRG_STAMP(1);

  // image space: byte j <-> stream byte g0 + j, g0 = wave_out rounded down to 16
  const uint32_t sh = static_cast<uint32_t>(wave_out & 15u);
  const uint64_t g0 = wave_out - sh;
  const uint32_t a0 = static_cast<uint32_t>(off - wave_out) + sh;  // this record's first byte
  const uint32_t span = sh + T;
  const uint32_t rounds = T ? (span + C - 1u) / C : 1u;
  const uint64_t ge = min<uint64_t>(wave_out + T, cap);  // last stream byte + 1 to write

  bool ok = szok;
  uint32_t M = 0;

  // one batch of payload chunks: U per lane, chunks c0 + 64 u + lane
  struct batch {
    u32x4 val[U];
    uint64_t hs[U];
    uint32_t at[U], nb[U], rm[U];
    bool fast[U];
    uint32_t tok;  // 0, defined after the asm loads (orders the stores after them)
  } B;
  B.tok = 0;
  // ASM: the loads as inline asm, which the compiler does not count: their
  // wait is the explicit one after the window's stores (XDRG_ENC_PIPE)
  auto issue = [&](uint32_t c0, uint32_t chi, batch &b, auto asm_tag) {
    uint32_t lo[U];
#pragma unroll
    for (int u = 0; u < U; ++u) lo[u] = 0;
    uint32_t ix[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ix[u] = min(c0 + 64u * u + lane, chi - 1u);
#pragma unroll
    for (uint32_t s = 32; s; s >>= 1) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (cum[lo[u] + s - 1u] <= ix[u]) lo[u] += s;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t rem = ix[u] - (lo[u] ? cum[lo[u] - 1u] : 0u);
      const echunk_desc *dl = desc + lo[u] * KMAX;
      echunk_desc d = dl[0];
#pragma unroll
      for (int k = 0; k + 1 < KMAX; ++k) {
        const uint32_t nq = (d.len + 15u) >> 4;
        if (rem >= nq) {
          rem -= nq;
          d = dl[k + 1];
        }
      }
      const bool live = c0 + 64u * u + lane < chi;
      const uint32_t q16 = rem << 4;
      b.hs[u] = d.src + q16;
      b.rm[u] = live ? d.len - q16 : 16u;
      b.at[u] = d.dst + q16;
      b.nb[u] = live ? min(16u, ((d.len + 3u) & ~3u) - q16) : 0u;
      b.fast[u] = live && b.hs[u] + 16u <= heap_len;
    }
    if constexpr (decltype(asm_tag)::value) {
      // every lane loads (a lane with no fast chunk: the heap's first 16
      // bytes -- the pipelined windows run only on heaps of 16 bytes or
      // more), so the batch is straight-line code before the stores and
      // their wait (tools/isa_audit.py).  (Dword-aligned loads of 16 bytes
      // plus the next word joined with v_alignbyte, in place of these
      // byte-misaligned ones: recvar 0.0998 vs 0.0957 ms, rpc 0.1385 vs
      // 0.1361, slower; profiles/r05h/ab_align.log.)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint8_t *pa = heap + (b.fast[u] ? b.hs[u] : 0ull);
        asm volatile("global_load_dwordx4 %0, %1, off ; xb1" : "=v"(b.val[u]) : "v"(pa));
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (b.fast[u]) {
          if constexpr ((XDRG_ENC_NT & 1) != 0) {
            b.val[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(heap + b.hs[u]));
          } else {
            b.val[u] = ld16u(heap + b.hs[u]);
          }
        }
    }
    if constexpr (decltype(asm_tag)::value) asm volatile("v_mov_b32 %0, 0" : "=v"(b.tok));
    __builtin_amdgcn_sched_barrier(0);
  };
  auto place = [&](batch &b, uint32_t w0) {
    // every load of the batch counts as consumed here, on every path (a
    // load left pending on some path makes the compiler wait for all
    // memory before the next write of these registers)
#pragma unroll
    for (int u = 0; u < U; ++u) asm volatile("" ::"v"(b.val[u]));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!b.nb[u]) continue;
      u32x4 x = b.val[u];
      if (!b.fast[u]) x = heap_tail16(heap, heap_len, b.hs[u]);
      const int32_t rr = static_cast<int32_t>(b.rm[u]);
      if (rr < 16) {  // zero the pad bytes after the payload (put_bytes)
        x.x &= keep_bytes(rr);
        x.y &= keep_bytes(rr - 4);
        x.z &= keep_bytes(rr - 8);
        x.w &= keep_bytes(rr - 12);
      }
      const uint32_t j = b.at[u] - w0;
      if (j + 16u <= C && b.at[u] >= w0) {
        uint32_t *wp = reinterpret_cast<uint32_t *>(img + j);
        wp[0] = x.x;
        if (b.nb[u] > 4u) wp[1] = x.y;
        if (b.nb[u] > 8u) wp[2] = x.z;
        if (b.nb[u] > 12u) wp[3] = x.w;
      } else {  // a chunk across a window edge
        c.wput(b.at[u], x.x);
        if (b.nb[u] > 4u) c.wput(b.at[u] + 4, x.y);
        if (b.nb[u] > 8u) c.wput(b.at[u] + 8, x.z);
        if (b.nb[u] > 12u) c.wput(b.at[u] + 12, x.w);
      }
    }
  };
  // pipelined windows (XDRG_ENC_PIPE): full windows leave as SW buffer
  // stores per lane; the wave's head chunk (shared with the previous wave's
  // stretch) is kept by lane 0 and written last, word by word
  constexpr uint32_t SW = CMAX / 1024u;
  constexpr bool kPipe = XDRG_ENC_PIPE && SW > 0 && (U == 2 || U == 4 || U == 8);  // vm_wait_after's shapes
  const bool pipe = kPipe && C <= CMAX && wave_out + T <= cap && heap_len >= 16;
  bool pf = false;
  u32x4 head = u32x4{0u, 0u, 0u, 0u};
  for (uint32_t rd = 0; rd < rounds; ++rd) {
    const uint32_t w0 = rd * C;
    c.w0 = w0;
    // ---- walk: the window's scalar words -> image, payload slots -> registers
    // (every lane walks in the first round: it reports the record's errors)
    if (PRE == 0 && (rd == 0 || (WL == 0 && ok && a0 < w0 + C && a0 + v > w0))) {
      c.at = a0;
      c.pos = off;
      bool okr = szok;
      if constexpr (NW > 0 && !RREG) {
        const uint32_t *t32 = reinterpret_cast<const uint32_t *>(tile + lane * stride);
#pragma unroll
        for (int k = 0; k < NW; ++k) rec[k] = t32[k];
        if constexpr (WL > 0) wave_sync();  // every tile read before the list (mark included) overwrites it
      }
      auto walk = [&](auto &cc, bool o) -> bool {
        if constexpr (NW > 0) {
          return w.enc(cc, reinterpret_cast<const uint8_t *>(rec), o);
        } else {
          return w.enc(cc, tile + lane * stride, o);
        }
      };
      bool checked = true;
      if constexpr (W::kFastWalk) {
        // the wave's bytes fit `cap` and the plan's depth fits the stack
        // budget: no field can fail a check -- walk without them
        if (wave_out + T <= cap && W::kMaxDepth <= stack_limit) {
          checked = false;
          enc_ctx<KMAX, false, WL> f = c.template as<false>();
          if (okr && mark) f.put(mark_word(sz - 4u));
          okr = walk(f, okr);
          c.take(f);
        }
      }
      if (checked) {
        if (okr && mark) {  // the message's record mark (message_t::alloc, marshal.cc:15-31)
          if (4 > cap - min(c.pos, cap)) {
            report(err, r, kOpRecordLevel, XDRG_ERR_OVERFLOW_PUT);
            okr = false;
          } else {
            c.put(mark_word(sz - 4u));
          }
        }
        okr = walk(c, okr);
      }
      if (rd == 0) {
        ok = okr;
        if (!ok) {  // a failing record's bytes are unspecified (never past `cap`)
#pragma unroll
          for (int k = 0; k < KMAX; ++k) c.pln[k] = 0;
        }
      }
    }
    if (rd == 0) {
      XDRG_STAMP(2);
      // ---- the lanes' slots and inclusive chunk counts, for the chunk pass
      uint32_t nch = 0;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        desc[lane * KMAX + k] = echunk_desc{c.psr[k], c.pds[k], c.pln[k]};
        nch += (c.pln[k] + 15u) >> 4;
      }
      const uint32_t ci = wave_incl_scan(nch);
      cum[lane] = ci;
      M = rl32(ci, 63);
      XDRG_STAMP(3);
    }
    wave_sync();
    if constexpr (WL > 0)
      if (ok && a0 < w0 + C && a0 + v > w0) emit_words(c, a0);

    // ---- payload chunks of the window: heap -> image, U per lane in flight.
    // Chunk i of the wave (stream order) belongs to the lane L with
    // cum[L-1] <= i < cum[L] (binary search) and to the first of its slots
    // whose chunks reach past i - cum[L-1].
    const uint32_t clo = rl32(wave_incl_scan(chunks_ending_by(c, w0)), 63);
    const uint32_t chi = min(M, rl32(wave_incl_scan(chunks_starting_before(c, w0 + C)), 63));
    uint32_t c0 = clo;
    if (pf) {  // this window's first batch was loaded during the last window's stores
      place(B, w0);
      c0 += 64u * U;
    }
    for (; c0 < chi; c0 += 64u * U) {
      issue(c0, chi, B, bool_tag<false>{});
      place(B, w0);
    }
    wave_sync();
    if (rd + 1 == rounds) XDRG_STAMP(4);

    // ---- window -> stream: aligned 16-byte chunks, words at the stretch's edges
    const uint64_t ws = g0 + w0;
    const uint64_t we = min<uint64_t>(ws + C, ge);
    pf = false;
    if (pipe && rd + 1 < rounds) {
      // a full window (we = ws + C): first the next window's first batch...
      const uint32_t w1 = w0 + C;
      const uint32_t nlo = rl32(wave_incl_scan(chunks_ending_by(c, w1)), 63);
      const uint32_t nhi = min(M, rl32(wave_incl_scan(chunks_starting_before(c, w1 + C)), 63));
      if (nlo < nhi) {
        issue(nlo, nhi, B, bool_tag<true>{});
        pf = true;
      }
      // ...then SW stores per lane, none skipped by a branch
      if (rd == 0 && sh && lane == 0) head = *reinterpret_cast<const u32x4 *>(img);
      const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(xdr + ws) >> 32));
      const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(xdr + ws)));
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void *>((static_cast<uint64_t>(hi) << 32) | lo), 0, C, 0x00020000);
      const uint32_t nc = C >> 4;
#pragma unroll
      for (uint32_t j = 0; j < SW; ++j) {
        const uint32_t k = lane + 64u * j;
        const bool drop = k >= nc || (rd == 0 && k == 0 && sh);
        const u32x4 v = *reinterpret_cast<const u32x4 *>(img + 16u * min(k, nc - 1u));
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (drop ? 0x80000000u : 16u * k) + B.tok, 0,
                                               (XDRG_ENC_NT & 2) != 0 ? 2 : 0);
      }
      // the prefetched loads were issued before these SW stores and vmcnt
      // retires in order: at most SW outstanding = every load has landed
      // (on every path, prefetched or not: tools/isa_audit.py's dataflow
      // then sees every batch waited for)
      vm_wait_after<SW>(B.val);
    } else if (we > ws) {
      const uint32_t nc = static_cast<uint32_t>((we - ws + 15u) >> 4);
      for (uint32_t k = lane; k < nc; k += 64u) {
        const uint64_t ca = ws + 16ull * k;
        const uint8_t *lsrc = img + 16u * k;
        if (ca >= wave_out && ca + 16u <= we) {
          if constexpr ((XDRG_ENC_NT & 2) != 0)
            __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(lsrc), reinterpret_cast<u32x4 *>(xdr + ca));
          else
            *reinterpret_cast<u32x4 *>(xdr + ca) = *reinterpret_cast<const u32x4 *>(lsrc);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const uint64_t wa = ca + 4u * t;
            if (wa >= wave_out && wa + 4u <= we) st32(xdr + wa, *reinterpret_cast<const uint32_t *>(lsrc + 4 * t));
          }
        }
      }
    }
    wave_sync();  // the next window's walk reuses the image
  }
  if (pipe && rounds > 1 && sh && lane == 0) {  // the head chunk's words of this wave
    if (sh <= 4) st32(xdr + g0 + 4, head.y);
    if (sh <= 8) st32(xdr + g0 + 8, head.z);
    st32(xdr + g0 + 12, head.w);
  }
  XDRG_STAMP(5);
}


// ---------------------------------------------------------------- decode
// LDS of a decode wave: the native tile (none when the walk decodes into
// registers, NWD > 0) and the window.
__host__ __device__ inline uint32_t dec_w_lds(uint32_t stride, uint32_t C, bool regs = false, uint32_t S = 0) {
  return (regs ? 0u : ((64u * stride + 15u) & ~15u)) + C + 32u + S;
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
    // word k (0..7) of the 32 bytes, by selects on its bits (a variable
    // vector index would put ra0/ra1 in scratch memory)
    const uint32_t k = static_cast<uint32_t>(ga - ra_line) >> 2;
    const bool b0 = k & 1u, b1 = k & 2u, b2 = k & 4u;
    const uint32_t x0 = b2 ? ra1.x : ra0.x, x1 = b2 ? ra1.y : ra0.y;
    const uint32_t x2 = b2 ? ra1.z : ra0.z, x3 = b2 ? ra1.w : ra0.w;
    return b1 ? (b0 ? x3 : x2) : (b0 ? x1 : x0);
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
  uint8_t *heap;  // decoded heap (element arrays live at [ecur, eend))
  uint64_t ecur, eend;
  bool zeroed = false;  // the arrays' bytes are zero already (the group's LDS stage)

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
  // the element area of a container of inline elements (elem_area_ok)
  __device__ __forceinline__ bool area(uint32_t op, uint32_t cnt, uint32_t stride, uint32_t wire) {
    if (elem_area_ok(ecur, eend, cnt, stride, wire, b - p)) return true;
    return fail(op, XDRG_ERR_OVERFLOW_GET);
  }
  // ... of an element subroutine's container: every element takes at least
  // `minw` wire bytes, so a count the bytes left cannot hold fails before
  // any element (sub_kernels.h, oracle/xdr_oracle.c)
  __device__ __forceinline__ bool area_sub(uint32_t op, uint32_t cnt, uint32_t stride, uint32_t minw) {
    ecur = (ecur + 7u) & ~7ull;
    const uint64_t bytes = static_cast<uint64_t>(cnt) * stride;
    if (static_cast<uint64_t>(cnt) * minw > b - p || ecur > eend || bytes > eend - ecur)
      return fail(op, XDRG_ERR_OVERFLOW_GET);
    return true;
  }
};


// NWD > 0 (plan-specialized walks, whose native offsets are constants): the
// lane decodes its record into NWD registers and stores them itself, so the
// wave keeps no native tile in LDS (more waves per CU, or a larger window).
template <class W, bool COPY, bool RA, int NWD = 0>
__device__ __forceinline__ void var_decode_body(
    const W &w, const uint8_t *__restrict__ xdr, uint64_t len, const uint64_t *__restrict__ offsets,
    uint64_t n, uint8_t *__restrict__ native, uint32_t stride, uint8_t *__restrict__ heap,
    uint32_t stack_limit, uint32_t C, uint64_t ebase, uint32_t F, uint32_t mark, uint32_t S,
    unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  const uint32_t lane = threadIdx.x;
  const uint32_t tile_bytes = NWD > 0 ? 0u : (64u * stride + 15u) & ~15u;
  uint8_t *tile = sm;
  uint8_t *win = sm + tile_bytes;
  uint8_t *stage = win + C + 32u;  // S bytes: the group's element arrays (packed plans)
  const uint64_t wr0 = static_cast<uint64_t>(blockIdx.x) * 64u;
  const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(64, n - wr0));
  const uint64_t r = wr0 + lane;
  XDRG_DSTAMP(0);
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
  XDRG_DSTAMP(1);

  for (uint32_t i = lane; i < tile_bytes / 16u; i += 64u)
    reinterpret_cast<u32x4 *>(tile)[i] = u32x4{0u, 0u, 0u, 0u};
  // The window: aligned 16-byte chunks covering [ws, ws + wc), 16 loads in
  // flight per lane, into LDS.  A chunk never leaves the pages that hold
  // stream bytes, so edge chunks load whole.  No global store is issued
  // before the walk: on gfx9 loads and stores share one counter, so a load
  // issued after a store would also wait for the store to complete.
  const uint32_t nwin = static_cast<uint32_t>((sh + wc + 15u) >> 4);
  const uint8_t *g0 = xdr + ws - sh;
  {
    constexpr int UL = 16;
    for (uint32_t c0 = 0; c0 < nwin; c0 += 64u * UL) {
      u32x4 v[UL];
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const uint32_t ci = c0 + 64u * u + lane;
        if (ci < nwin) v[u] = *reinterpret_cast<const u32x4 *>(g0 + 16u * ci);
      }
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const uint32_t ci = c0 + 64u * u + lane;
        if (ci < nwin) reinterpret_cast<u32x4 *>(win)[ci] = v[u];
      }
    }
  }
  wave_sync();
  XDRG_DSTAMP(2);

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
  c.eend = ebase + static_cast<uint64_t>(F) * b;
  // ... packed with the group's (packed_area).  When the group's arrays fit
  // the stage (S bytes of LDS) the walk writes them there and the wave
  // stores them after it as whole lines: written straight from the walk,
  // each lane's stores land in lines its neighbours fill at other steps of
  // the walk, and L2 evicts many of them half-written (vecrec: 350 MiB
  // written per launch for ~280 MiB of data, profiles/r03p).
  uint64_t ga = 0, gtot = 0;  // the group's arrays: [ga, ga + gtot)
  bool staged = false;
  if (w.packed()) {
    const bool bad = lane < nrec && (b < a || b > len);
    const bool on = lane < nrec && !bad && a + mark <= b;
    const uint64_t e = w.ebytes(c.rd, a + mark, b, on);
    const uint64_t E = on ? min(e, ebudget(F, a, b)) : 0u;
    ga = packed_area(E, bad, rl64(a, 0), ebase, F, c.ecur, c.eend);
    gtot = rl64(c.eend, 63) - ga;
    staged = gtot <= S;
    if (staged) {  // zeroed: the stage leaves whole, gaps and all
      for (uint32_t i = lane; i < (gtot + 15u) / 16u; i += 64u)
        reinterpret_cast<u32x4 *>(stage)[i] = u32x4{0u, 0u, 0u, 0u};
      wave_sync();
    }
  }
  uint32_t rec[NWD > 0 ? NWD : 1];
#pragma unroll
  for (int k = 0; k < (NWD > 0 ? NWD : 1); ++k) rec[k] = 0u;
  {
    uint8_t *nat = NWD > 0 ? reinterpret_cast<uint8_t *>(rec) : tile + lane * stride;
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
    if (staged) {  // the same walk, its arrays into the stage
      c.heap = stage - ga;
      c.zeroed = true;
      ok = w.dec(c, nat, ok);
    } else {
      ok = w.dec(c, nat, ok);
    }
    if (ok && c.p != b) report(err, r, kOpRecordLevel, XDRG_ERR_TRAILING);
  }
  wave_sync();
  if (staged) {  // [ga, ga + gtot): 8-aligned, a multiple of 8 bytes; whole lines, not
                 // re-read here: non-temporal (vecrec 0.138 -> 0.128 ms, profiles/r03s)
    const uint64_t *src = reinterpret_cast<const uint64_t *>(stage);
    uint64_t *dst = reinterpret_cast<uint64_t *>(heap + ga);
    for (uint32_t i = lane; i < gtot / 8u; i += 64u) __builtin_nontemporal_store(src[i], dst + i);
  }
  XDRG_DSTAMP(3);
  if (COPY) {
    // The decoded heap is the stream: the stretch [ws, we) to heap + ws.
    // Chunks past the window are loaded first (all in flight), then the
    // window's chunks leave from LDS, then those.
    const uint64_t nall = (sh + (we - ws) + 15u) >> 4;
    const int64_t lim = static_cast<int64_t>(we - ws);
    uint8_t *h0 = heap + ws - sh;
    auto put = [&](uint64_t ci, const u32x4 &x) {
      const int64_t o = static_cast<int64_t>(16u * ci) - sh;  // stream offset - ws
      if (o >= 0 && o + 16 <= lim) {
        if constexpr (XDRG_DEC_NT)
          __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(h0 + 16u * ci));
        else
          st16u(h0 + 16u * ci, x);
      } else {
        uint8_t *hd = h0 + 16u * ci;
        if (o >= 0 && o + 4 <= lim) st32(hd, x.x);
        if (o + 4 >= 0 && o + 8 <= lim) st32(hd + 4, x.y);
        if (o + 8 >= 0 && o + 12 <= lim) st32(hd + 8, x.z);
        if (o + 12 >= 0 && o + 16 <= lim) st32(hd + 12, x.w);
      }
    };
    constexpr int UB = 8;
    for (uint64_t c0 = nwin; c0 < nall || c0 == nwin; c0 += 64u * UB) {
      u32x4 v[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const uint64_t ci = c0 + 64u * u + lane;
        if (ci < nall) v[u] = *reinterpret_cast<const u32x4 *>(g0 + 16u * ci);
      }
      if (c0 == nwin)
        for (uint32_t ci = lane; ci < nwin; ci += 64u) put(ci, reinterpret_cast<const u32x4 *>(win)[ci]);
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const uint64_t ci = c0 + 64u * u + lane;
        if (ci < nall) put(ci, v[u]);
      }
      if (c0 + 64u * UB >= nall) break;
    }
  }
  uint8_t *ndst = native + wr0 * stride;
  if constexpr (NWD > 0) {
    if (lane < nrec) {
      uint8_t *d = ndst + lane * stride;
      if constexpr (NWD % 4 == 0) {
#pragma unroll
        for (int k = 0; k < NWD; k += 4)
          *reinterpret_cast<u32x4 *>(d + 4 * k) = u32x4{rec[k], rec[k + 1], rec[k + 2], rec[k + 3]};
      } else if constexpr (NWD % 2 == 0) {
#pragma unroll
        for (int k = 0; k < NWD; k += 2)
          *reinterpret_cast<unsigned long long *>(d + 4 * k) =
              static_cast<unsigned long long>(rec[k]) | (static_cast<unsigned long long>(rec[k + 1]) << 32);
      } else {
#pragma unroll
        for (int k = 0; k < NWD; ++k) st32(d + 4 * k, rec[k]);
      }
    }
  } else {
    const uint32_t nbytes = nrec * stride;
    for (uint32_t i = lane; i < nbytes / 16u; i += 64u)
      reinterpret_cast<u32x4 *>(ndst)[i] = reinterpret_cast<const u32x4 *>(tile)[i];
    for (uint32_t i = (nbytes / 16u) * 4u + lane; i < nbytes / 4u; i += 64u)
      reinterpret_cast<uint32_t *>(ndst)[i] = reinterpret_cast<const uint32_t *>(tile)[i];
  }
  XDRG_DSTAMP(4);
}

// ------------------------------------------------------------------ size
// One 64-thread workgroup = 64 consecutive records, natives staged in LDS
// with coalesced 16-byte loads -- or, with NW (the record's words, a
// generated walk whose field offsets are constants), each lane's record
// loaded straight into registers as var_encode_body's load_rec does, all of
// its loads in flight at once and no LDS round trip.  sizes[r] = xdr_size
// (kSizeErr on a bad discriminant, reported as the size pass of k_var_size
// does), block_sums = the 64-record sums.
template <class W, int NW = 0>
__device__ __forceinline__ void var_size_body(const W &w, const uint8_t *__restrict__ native, uint64_t n,
                                              uint32_t stride, const uint8_t *__restrict__ heap,
                                              uint64_t heap_len, uint32_t *__restrict__ sizes,
                                              unsigned long long *__restrict__ block_sums,
                                              uint32_t mark, unsigned long long *err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
  const uint32_t lane = threadIdx.x;
  const uint64_t wr0 = static_cast<uint64_t>(blockIdx.x) * 64u;
  const uint64_t r = wr0 + lane;
  const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(64, n - wr0));
  const uint8_t *nsrc = native + wr0 * stride;
  constexpr uint32_t kAl = NW % 4 == 0 ? 16u : NW % 2 == 0 ? 8u : 4u;
  const bool regs = NW > 0 && stride == 4u * NW && (reinterpret_cast<uintptr_t>(native) & (kAl - 1)) == 0;
  uint32_t rec[NW > 0 ? NW : 1];
  if (regs) {
#pragma unroll
    for (int k = 0; k < (NW > 0 ? NW : 1); ++k) rec[k] = 0u;
    if (lane < nrec) {
      const uint8_t *src = nsrc + static_cast<uint64_t>(lane) * stride;
      if constexpr (NW % 4 == 0) {
#pragma unroll
        for (int k = 0; k < NW; k += 4) {
          const u32x4 q = *reinterpret_cast<const u32x4 *>(src + 4 * k);
          rec[k] = q.x; rec[k + 1] = q.y; rec[k + 2] = q.z; rec[k + 3] = q.w;
        }
      } else if constexpr (NW % 2 == 0) {
#pragma unroll
        for (int k = 0; k < NW; k += 2) {
          const uint2 q = *reinterpret_cast<const uint2 *>(src + 4 * k);
          rec[k] = q.x; rec[k + 1] = q.y;
        }
      } else {
#pragma unroll
        for (int k = 0; k < (NW > 0 ? NW : 1); ++k) rec[k] = ld32(src + 4 * k);
      }
    }
  } else {
    if ((reinterpret_cast<uintptr_t>(nsrc) & 15u) == 0) {
      stage_tile<8>(tile, nsrc, nrec * stride, lane, 64u);
    } else {
      for (uint32_t i = lane; i < nrec * stride / 4u; i += 64u)
        reinterpret_cast<uint32_t *>(tile)[i] = reinterpret_cast<const uint32_t *>(nsrc)[i];
    }
    wave_sync();
  }
  uint32_t size = 0;
  if (r < n) {
    uint32_t bad_op = 0xffffffffu;
    // (two calls, not one through a selected pointer: the register copy stays
    // registers only when its walk sees the array itself)
    const uint64_t s = (regs ? w.size(reinterpret_cast<const uint8_t *>(rec), heap, heap_len, bad_op)
                             : w.size(tile + lane * stride, heap, heap_len, bad_op)) + mark;
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
