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
// (a generated parse over a staged stretch: the record runs past the stretch)
constexpr uint32_t RX_OUT = 0xfffffffdu;

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

// Stream words for a record parse: straight from global memory, or from a
// stretch staged in LDS (global past it).  Every read is of a 4-byte word
// at a 4-aligned offset inside the stream (the parse checks the bound
// before it reads).
// Readers.  Generated parses (codegen.cpp rx_block) call clamp() on their
// bound once and then read with at(), unchecked: every read lies inside the
// bound tested before it.
struct rx_global {
  const uint8_t *s;
  __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return ld32(s + p); }
  __device__ __forceinline__ uint32_t at(uint64_t p) const { return ld32(s + p); }
  template <class U>
  __device__ __forceinline__ void clamp(U &, uint32_t &, U) const {}
};
// The fast path (rxs_*) parses in 32-bit offsets from the start of its
// staged stretch: rx_lds reads the stretch alone -- a read outside it sets
// `out` (and reads word 0) and the caller parses that record again with
// rx_goff, from global memory.  Keeping the two apart matters: one reader
// choosing between LDS and global per read compiles to flat loads, which
// take the vector memory path for LDS too.
struct rx_lds {
  const uint32_t *w;  // LDS: the stretch's first nb bytes
  uint32_t nb;
  mutable bool out;
  __device__ __forceinline__ uint32_t operator()(uint32_t p) const {
    uint32_t d = p;
    if (d >= nb) { out = true; d = 0; }
    return w[d >> 2];
  }
  // a bound past the stretch becomes its end, and a parse that reaches it
  // ends RX_OUT (a value test before that fails the same way from global).
  // A bound that is not a whole number of words from a (an odd maxlen, a
  // ragged stream end) sends the record to global memory at once: a payload
  // tested unpadded may then end up to 3 bytes past the bound, and the
  // tests after it wrap (the decode's own behaviour, which only the
  // checked reads reproduce).
  __device__ __forceinline__ uint32_t at(uint32_t p) const { return w[p >> 2]; }
  // (rlen_st: a failed record's reads go on, held inside the stretch)
  __device__ __forceinline__ uint32_t atc(uint32_t p) const { return w[min(p, nb >= 4u ? nb - 4u : 0u) >> 2]; }
  __device__ __forceinline__ void clamp(uint32_t &lim, uint32_t &past, uint32_t a) const {
    if (lim > nb || ((lim - a) & 3u)) {
      lim = ((lim - a) & 3u) ? a : nb;
      past = RX_OUT;
    }
  }
};
struct rx_goff {
  const uint8_t *b;  // the stretch's start in global memory
  __device__ __forceinline__ uint32_t operator()(uint32_t p) const { return ld32(b + p); }
  __device__ __forceinline__ uint32_t at(uint32_t p) const { return ld32(b + p); }
  template <class U>
  __device__ __forceinline__ void clamp(U &, uint32_t &, U) const {}
};
// ---------------------------------- speculative record index (fast path)
// xdrg_index_records' list ranking parses every word of the stream as a
// possible record start.  The fast path parses (almost) only the records
// themselves, speculating where each piece of the stream is entered and
// checking every guess exactly:
//   rxs_walk   one wave per kRxsSeg-byte segment, staged in LDS with the
//              kRxsBack bytes before it and kRxsAhead after.  Lane j takes
//              kRxsSub bytes, the first lanes the look-back: its guess is the
//              first word from which a chain of record parses runs past the
//              lane's end.  The lanes then agree from lane 0 on (each
//              re-walks from its predecessor's exit until no exit changes),
//              so the chain enters the segment proper (lane kRoot) from a guess
//              a kilobyte before it, by then usually the true chain: its
//              first node there is the segment's entry E.  The segment's
//              lanes count their nodes and write them out (segment-relative
//              words, u16).
//   rxs_check  per segment: the previous segment's exit (the true chain's
//              first node at or past this segment's start) must be E, or a
//              later node of this segment where a chain that entered early
//              merged into the true one, and no chain may break; the nodes
//              from it on are the segment's records.  (A record that spans
//              a whole segment passes only when the guess agrees.)  In a
//              walk over records of any length (WHOLE) a segment that fails
//              goes to rxs_fix instead.
//   rxs_fix    (WHOLE) one wave re-decides the failed segments in stream
//              order from the true entry (below).
//   (scan)     exclusive scan of those counts (launch_block_scan).
//   rxs_emit   when the last exit is the stream's end and the chain holds
//              exactly n records: offsets[] from the node lists, offsets[n]
//              and the count, and the flag says so; else the flag sends the
//              batch down the list ranking.
// Any stream the fast path does not take (a damaged one, trailing records,
// a record longer than the window, a guess that missed) therefore gets the
// list ranking's exact answer; tests/test_record_index.py checks both on
// the same streams.
// 63 words per lane would start lane j's stretch at LDS bank -j (mod 32),
// so the lanes' reads at like offsets hit 32 different banks (ds_read_b32
// banks by (a/4) mod 32 over each half-wave; with 64 words per lane every
// lane of a half-wave reads the same bank, a 32-way conflict, measured).
// 31 words per lane does the same (31j = -j mod 32), and its 9 KiB stretch
// per wave lets 17 waves share a CU's LDS (latency hiding for the walks,
// which are chains of dependent LDS reads) where 63 words (17 KiB) let 9
constexpr uint32_t kRxsSub = 124;                         // bytes per lane
constexpr uint32_t kRxsBackLanes = 8;                     // look-back: lanes 0-7 (992 bytes)
constexpr uint32_t kRxsBack = kRxsBackLanes * kRxsSub;
constexpr uint32_t kRxsSeg = 64 * kRxsSub - kRxsBack;     // bytes per segment (one wave): lanes 8-63
constexpr uint32_t kRxsAhead = 9u * 1024 - 64 * kRxsSub;  // staged past the segment (1280)
constexpr uint64_t kRxsBroken = ~0ull;
// in the walk (32-bit offsets into the stretch): a broken chain, no state
constexpr uint32_t kBrk = 0xffffffffu, kNone = 0xfffffffeu;
// segment record: entry E, exit, node count (kRxsBroken: the chain broke),
// and (rxs_check / rxs_fix) the index of its first true node
constexpr uint32_t kRxsSegWords = 4;

// One record parse at q: from the staged stretch, or from global memory
// when the record reaches past it.  In a walk over a stream of records of
// any length (WHOLE: xdrg_index_records with max_rec_len past the index
// window) such a record is RX_OUT: it is left to the wave, which parses it
// at the walk's end through blocks of the stream in LDS (one lane's parse through
// global memory waits on every length it reads: a 500-node rp__list took
// milliseconds that way), and the walk knows where it starts -- a record
// from the look-back that runs past the stretch is the segment's only
// when the segment lies inside it (below), while a guess there that reads
// a large word as a length would otherwise carry the chain far away.
template <bool WHOLE = false, class P>
__device__ __forceinline__ uint32_t rxs_rlen(const P &parser, const uint32_t *smem, const rx_lds &st,
                                             const uint8_t *base, uint32_t lenr, uint32_t maxlen, uint32_t q) {
  st.out = false;
  const uint32_t L = parser.rlen_st(smem, st, lenr, q, maxlen);
  if (!st.out && L != RX_OUT) return L;
  if constexpr (WHOLE) return RX_OUT;
  return parser.rlen_rd(smem, rx_goff{base}, lenr, q, maxlen);
}

// The nodes a walk passes, kept for the node list: the first kRxsKeep (as
// stretch offsets) and how many there were (more: the list is walked again).
constexpr uint32_t kRxsKeep = 6;
struct rxs_nodes {
  uint32_t n = 0;
  uint32_t w[kRxsKeep];
  __device__ __forceinline__ void add(uint32_t q) {
#pragma unroll
    for (uint32_t i = 0; i < kRxsKeep; ++i) w[i] = n == i ? q : w[i];
    ++n;
  }
};

// Chain of record parses from q until it reaches b, noting its nodes: the
// position reached, or kBrk -- or (WHOLE) kLongAt | q for a chain whose
// record at q runs past the staged stretch: it passes every lane after it
// (kLongAt | q is at or past any lane's end) and becomes the segment's
// exit, which the wave resolves to the record's end (rx_blk).
constexpr uint32_t kLongAt = 0x80000000u;  // (stretch offsets stay below 2^31)
template <bool WHOLE = false, class P>
__device__ __forceinline__ uint32_t rxs_chain(const P &parser, const uint32_t *smem, const rx_lds &st,
                                              const uint8_t *base, uint32_t lenr, uint32_t maxlen, uint32_t q,
                                              uint32_t b, rxs_nodes &nd) {
  nd.n = 0;
  while (q < b) {
    nd.add(q);
    const uint32_t L = rxs_rlen<WHOLE>(parser, smem, st, base, lenr, maxlen, q);
    if (WHOLE && L == RX_OUT) return kLongAt | q;
    if (L >= RX_LONG) return kBrk;
    q += L;
  }
  return q;
}

// The "parse" of a record mark (RFC 5531) for the walk over a message
// stream (xdrg_index_msgs): a mark whose message read_message takes
// (srpc.cc:29-55: the pre-swap size test, the last-fragment bit, a size
// within maxmsglen_ and the stream, a multiple of 4 for xdr_from_msg) is a
// record of 4 + size bytes; anything else ends the chain, and the list
// ranking then classifies it as read_message would (ix_mark).
struct mark_rx {
  uint32_t maxlen;
  __device__ __forceinline__ void init(uint32_t *) const {}
  __device__ __forceinline__ bool first_ok(const uint32_t *, uint32_t v) const {
    const uint32_t size = v & ~XDRG_MARK_LAST;
    return !((v >> 24) & 3u) && (v & XDRG_MARK_LAST) && size <= maxlen && !(size & 3u);
  }
  // least bytes the record needs after its first checked word (the speculative
  // walk's second filter; first_ok already holds the size to maxlen)
  __device__ __forceinline__ uint64_t first_len(uint32_t) const { return 0; }
  __device__ __forceinline__ bool second_ok(uint32_t, uint32_t) const { return true; }
  __device__ __forceinline__ uint32_t rlen_st(const uint32_t *m, const rx_lds &rd, uint32_t len, uint32_t a,
                                              uint32_t maxlen) const {
    return rlen_rd(m, rd, len, a, maxlen);
  }
  template <class RD, class U>
  __device__ __forceinline__ uint32_t rlen_rd(const uint32_t *, const RD &rd, U len, U a, uint32_t) const {
    if (len - a < 4) return RX_BAD;
    const uint32_t raw = rd(a);
    const uint32_t v = bswap32(raw), size = v & ~XDRG_MARK_LAST;
    if ((raw & 3u) || !(v & XDRG_MARK_LAST) || size > maxlen || (size & 3u) || len - a - 4 < size) return RX_BAD;
    return 4u + size;
  }
};

// Phase timestamps for tools/tune/ix_stamps.py, which compiles a copy of a
// plan's generated source with this defined; nothing in the library does.
#ifndef XDRG_XSTAMP
#define XDRG_XSTAMP(k) ((void)0)
#endif
// ... and per-lane values of the guess phase (clock reads and counts)
#ifndef XDRG_LSTAMP
#define XDRG_LSTAMP(k, v) ((void)0)
#define XDRG_LCLK() 0ull
#endif
// ... and per-lane states of the walk (tools/gpu/rx_whole_diag.py)
#ifndef XDRG_LDBG
#define XDRG_LDBG(k, v) ((void)0)
#endif

// A WHOLE walk's chain whose last record runs past the staged stretch: the
// wave parses that record through kRxsLongBlk-byte blocks of the stream in
// LDS (the stretch's, free by then), each refilled by one round trip of the
// wave's 16-byte loads -- the same parse on every lane.
constexpr uint32_t kRxsLongBlk = 4096;
// Wave-uniform block reader (every lane asks for the same word).
struct rx_blk {
  const uint8_t *s;
  uint64_t len;
  uint32_t *buf;  // kRxsLongBlk bytes of LDS
  mutable uint64_t base;
  __device__ void load(uint64_t p) const {
    base = p & ~15ull;
    wave_sync();  // every lane has read the old block
    const uint32_t lane = __lane_id();
#pragma unroll
    for (uint32_t k = 0; k < kRxsLongBlk / 1024u; ++k) {
      const uint64_t o = base + 16u * lane + 1024u * k;
      u32x4 t;
      if (o + 16u <= len) {
        t = ld16u(s + o);
      } else {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = o + 4u * j + 4u <= len ? ld32(s + o + 4u * j) : 0u;
        t = u32x4{w[0], w[1], w[2], w[3]};
      }
      reinterpret_cast<u32x4 *>(buf)[lane + 64u * k] = t;
    }
    wave_sync();
  }
  __device__ __forceinline__ uint32_t at(uint64_t p) const {
    if (p - base >= kRxsLongBlk - 3u) load(p);
    return buf[(p - base) >> 2];
  }
  __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return at(p); }
  __device__ __forceinline__ uint32_t atc(uint64_t p) const { return at(p); }
  template <class U>
  __device__ __forceinline__ void clamp(U &, uint32_t &, U) const {}
};


template <bool WHOLE = false, class P>
__device__ __forceinline__ void rxs_walk_body(const P &parser, const uint8_t *__restrict__ s, uint64_t len,
                                              uint32_t maxlen, uint64_t *__restrict__ seg,
                                              uint16_t *__restrict__ nodes, uint32_t *__restrict__ flag,
                                              bool has_first, uint32_t fd) {
  constexpr uint32_t kStg = kRxsBack + kRxsSeg + kRxsAhead;
  constexpr uint32_t kRoot = kRxsBack / kRxsSub;  // first lane of the segment proper
  __shared__ __attribute__((aligned(16))) uint32_t stg[kStg / 4];
  extern __shared__ __attribute__((aligned(16))) uint32_t rx_smem[];
  const uint32_t lane = threadIdx.x;
  XDRG_XSTAMP(0);
  const uint64_t s0 = static_cast<uint64_t>(blockIdx.x) * kRxsSeg;
  const uint64_t lo = s0 >= kRxsBack ? s0 - kRxsBack : 0;
  const uint8_t *base = s + lo;
  // offsets from lo from here on (a record parse never looks past
  // maxlen, so the clamp changes nothing)
  const uint32_t lenr = static_cast<uint32_t>(min(len - lo, 0x7fffffffull));
  const uint32_t r0 = static_cast<uint32_t>(s0 - lo), r1 = static_cast<uint32_t>(min(len, s0 + kRxsSeg) - lo);
  if (blockIdx.x == 0 && lane == 0) {
    flag[0] = 1u;  // rxs_check clears it on a miss
    flag[2] = 0u;  // (WHOLE: the count of rxs_fix's list, a u64 at flag + 2)
    flag[3] = 0u;
  }
  parser.init(rx_smem);
  // stage [lo, lo + kStg) within the stream: all of a lane's 16-byte loads
  // in flight before its stores
  const uint32_t nb = min(lenr, kStg) & ~3u;
  {
    constexpr int U = kStg / 1024;
    u32x4 t[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t o = 16u * lane + 1024u * k;
      if (o + 16 <= nb) {
        t[k] = ld16u(base + o);
      } else {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = o + 4 * j + 4 <= nb ? ld32(base + o + 4 * j) : 0u;
        t[k] = u32x4{w[0], w[1], w[2], w[3]};
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) reinterpret_cast<u32x4 *>(stg)[lane + 64u * k] = t[k];
  }
  wave_sync();
  XDRG_XSTAMP(1);
  const rx_lds st{stg, nb, false};
  // lane j: [a, b); lanes below kRoot cover the look-back (none in the
  // first segment, whose chain starts at byte 0: lane kRoot is its root)
  const bool first = s0 == 0;
  const uint32_t root = first ? kRoot : 0;
  const uint32_t a = r0 + kRxsSub * lane - kRxsBack;  // (wraps for the first segment's look-back: inactive)
  const uint32_t b = min(a + kRxsSub, r1);
  const bool act = lane >= root && a < r1;
  // the lane's guess: g (its chain's first node), e (where it leaves the
  // lane), nd (its nodes)
  uint32_t g = kNone, e = kNone;
  rxs_nodes nd;
  [[maybe_unused]] const uint64_t lt0 = XDRG_LCLK();
  [[maybe_unused]] uint64_t lt1 = lt0;
  [[maybe_unused]] uint32_t ltry = 0;
  if (act && first && lane == root) {
    g = 0;
    e = rxs_chain<WHOLE>(parser, rx_smem, st, base, lenr, maxlen, 0, b, nd);
  } else if (act) {
    // candidates: the lane's words (before b, with a first checked word
    // inside the stream) whose first checked word passes; the lane's LDS reads
    // are issued before the tests (one round trip per 15, not per word)
    const uint32_t nk = (b - a + 3) / 4;
    const uint32_t nf = a + fd + 4 <= lenr ? (lenr - a - fd - 4) / 4 + 1 : 0u;
    const uint32_t nv = min(nk, nf);
    const uint64_t vmask = nv >= 64 ? ~0ull : (1ull << nv) - 1;
    uint64_t mask = vmask;
    if (has_first && fd <= 1024) {  // (fd > 1024: every word is a candidate)
      const uint32_t i0 = (a + fd) >> 2;  // + kRxsSub / 4 + 1 stays inside stg for fd <= 1024
      uint32_t fw[kRxsSub / 4 + 1];  // (+ the word after the last, for second_ok)
#pragma unroll
      for (uint32_t k = 0; k < kRxsSub / 4 + 1; ++k) fw[k] = stg[i0 + k];
      uint64_t m = 0;
      // a candidate must also fit its first field's least bytes in maxlen: a
      // record that cannot breaks the chain anyway (the walk then falls back
      // to the list ranking, which tells INDEX_LONG apart); containertest's
      // unbounded uvec<> and strings otherwise let every word through
      // (and in the rest of the stream: with no maxlen -- WHOLE -- that
      // spares the global parse of candidates whose first length cannot fit)
      const uint64_t room = min<uint64_t>(maxlen > fd + 4u ? maxlen - fd - 4u : 0u,
                                          lenr > a + fd + 4u ? lenr - a - fd - 4u : 0u);
#pragma unroll
      for (uint32_t k = 0; k < kRxsSub / 4; ++k) {
        const uint32_t v = bswap32(fw[k]);
        m |= static_cast<uint64_t>(parser.first_ok(rx_smem, v) && parser.first_len(v) <= room &&
                                   parser.second_ok(v, bswap32(fw[k + 1])))
             << k;
      }
      // words whose first checked word (or the one after it, second_ok's) is
      // past the staged stretch stay candidates
      const uint32_t ns = a + fd + 4 < nb ? (nb - a - fd - 4) / 4 : 0u;
      if (ns < 64) m |= ~0ull << ns;
      mask &= m;
    }
    lt1 = XDRG_LCLK();
    // (WHOLE: a chain that ends in a record past the stretch is the guess
    // only when no other candidate's chain leaves the lane: a word read as
    // a large length -- rp__list's 100000-based r_prog under a string's
    // length -- carries a wrong guess far into the stream)
    uint32_t gl = kNone, el = kNone;
    rxs_nodes ndl;
    while (mask) {
      const uint32_t k = __builtin_ctzll(mask);
      mask &= mask - 1;
      ++ltry;
      const uint32_t p = a + 4 * k;
      const uint32_t q = rxs_chain<WHOLE>(parser, rx_smem, st, base, lenr, maxlen, p, b, nd);
      if (WHOLE && q != kBrk && (q & kLongAt)) {
        if (gl == kNone) {
          gl = p;
          el = q;
          ndl = nd;
        }
        continue;
      }
      if (q != kBrk) { g = p; e = q; break; }
    }
    if (WHOLE && g == kNone && gl != kNone) {
      g = gl;
      e = el;
      nd = ndl;
    }
    if (g == kNone) nd.n = 0;
  }
  XDRG_LSTAMP(0, lt1 - lt0);
  XDRG_LSTAMP(1, XDRG_LCLK() - lt1);
  XDRG_LSTAMP(2, ltry);
  XDRG_LSTAMP(3, nd.n);
  if (lane == root && g == kNone) e = kBrk;  // a root without a chain
  XDRG_LDBG(0, g);
  XDRG_LDBG(1, e);
  XDRG_XSTAMP(2);
  // Agree from the root on.  A lane without a guess is transparent: no
  // word of it starts a chain that leaves it, so the chain either passes
  // over it (an entry at or past its end) or breaks there.  Every other
  // lane takes its entry from the nearest such lane before it (through the
  // transparent ones) and re-walks from it when it is not its guess; lanes
  // are final in order, one lane with a state per round.  In the look-back
  // a chain that breaks gives way to the lane's own guess (a wrong guess
  // upstream must not sink the segment); in the segment proper it breaks
  // the segment.
  const bool stateful = act && (g != kNone || lane == root);
  const uint64_t smask = __ballot(stateful);
  const uint64_t below = smask & ((1ull << lane) - 1);
  const uint32_t src = below ? 63u - static_cast<uint32_t>(__builtin_clzll(below)) : lane;
  const uint32_t g0 = g, e0 = e;
  const rxs_nodes nd0 = nd;
  uint32_t pin = g;  // the entry the lane's state follows from
  auto entry = [&](uint32_t pe) { return pe == kBrk || pe < a ? kBrk : pe; };
  const uint64_t below_seg = ((1ull << lane) - 1) & ~((1ull << kRoot) - 1);  // lanes [kRoot, lane)
  for (int it = 0; it < 64; ++it) {
    const uint32_t pe = entry(__shfl(e, src, 64));
    // a broken chain gives way to the lane's own guess in the look-back, and
    // in the segment proper until the segment's chain has started (a message
    // or record longer than the look-back can leave it without a chain); the
    // node list stays one chain, and rxs_check decides whether it is the true one
    const uint64_t livem = __ballot(stateful && lane >= kRoot && e != kBrk && e != kNone);
    bool ch = false;
    if (stateful && lane > root && pe != pin) {
      ch = true;
      pin = g = pe;
      nd.n = 0;
      e = pe == kBrk || pe >= b ? pe : rxs_chain<WHOLE>(parser, rx_smem, st, base, lenr, maxlen, pe, b, nd);
      // An entry from a look-back lane at or past the segment's end is one
      // record from the look-back over the whole segment: a true one puts
      // the segment inside it (rxs_check passes it over, whatever the walk
      // says), so it gives way to the lane's own guess like a broken chain
      // -- a wrong guess upstream that reads a large length (or a record
      // left to the wave's long parse, kLongAt) must not sink the segment
      const bool far = src < kRoot && pe != kBrk && pe >= r1;
      if ((e == kBrk || far) && g0 != kNone && (lane < kRoot || far || !(livem & below_seg))) {
        g = g0;
        e = e0;
        nd = nd0;
      }
    }
    if (!__any(ch)) break;
  }
  const uint32_t pt = entry(__shfl(e, src, 64));
  if (act && !stateful) {  // a transparent lane passes the chain over or breaks it
    g = pt;
    e = g == kBrk || g < b || (src < kRoot && g >= r1) ? kBrk : g;  // (a look-back record over the segment: above)
    nd.n = 0;
  }
  XDRG_LDBG(2, g);
  XDRG_LDBG(3, e);
  XDRG_XSTAMP(3);
  // the segment's nodes, noted by the walk that set each lane's state (the
  // look-back lanes' nodes belong to the segment before); a lane with more
  // than kRxsKeep walks again
  const bool live = act && lane >= kRoot && e != kBrk;
  const uint32_t c = live ? nd.n : 0u;
  XDRG_XSTAMP(4);
  const uint32_t incl = wave_incl_scan(c);
  uint16_t *out = nodes + static_cast<uint64_t>(blockIdx.x) * (kRxsSeg / 4) + (incl - c);
  if (live) {
#pragma unroll
    for (uint32_t i = 0; i < kRxsKeep; ++i)
      if (i < c) out[i] = static_cast<uint16_t>((nd.w[i] - r0) >> 2);
    if (c > kRxsKeep) {
      uint32_t q = g;
      for (uint32_t k = 0; k < c; ++k) {
        if (k >= kRxsKeep) out[k] = static_cast<uint16_t>((q - r0) >> 2);
        q += rxs_rlen<WHOLE>(parser, rx_smem, st, base, lenr, maxlen, q);  // (the last: RX_OUT, unused)
      }
    }
  }
  XDRG_XSTAMP(5);
  // the segment's exit: the last active lane's; E: the chain's first node
  // at or past s0 = the entry of the first lane of the segment proper with
  // a live state
  const uint64_t amask = __ballot(act);
  const uint32_t last = 63u - static_cast<uint32_t>(__builtin_clzll(amask));
  // (WHOLE: lanes passed over by a record left to the long parse hold no node)
  const bool passed = WHOLE && g != kBrk && g != kNone && (g & kLongAt);
  const uint64_t livef = __ballot(act && lane >= kRoot && e != kBrk && e != kNone && !passed);
  const uint32_t fl = livef ? static_cast<uint32_t>(__builtin_ctzll(livef)) : kRoot;
  const uint32_t x = __shfl(e, last, 64), E = __shfl(g, fl, 64);
  uint64_t xe = x == kBrk ? kRxsBroken : lo + (x & ~kLongAt);
  if constexpr (WHOLE) {
    if (x != kBrk && (x & kLongAt)) {  // (x is the wave's: every lane parses)
      const rx_blk rd{s, len, stg, 0};
      rd.load(xe);  // (its wave_sync: every lane is past its reads of the stretch)
      const uint32_t L = parser.template rlen_rd<rx_blk, uint64_t>(rx_smem, rd, len, xe, maxlen);
      xe = L >= RX_OUT ? kRxsBroken : xe + L;
    }
  }
  if (lane == 0) {
    uint64_t *r = seg + static_cast<uint64_t>(blockIdx.x) * kRxsSegWords;
    r[0] = !livef || E == kBrk ? kRxsBroken : lo + E;
    r[1] = xe;
    r[2] = x == kBrk ? kRxsBroken : rl32(incl, 63);
  }
}

// The true entry among segment i's nodes (nodes ascend: binary search): its
// index, or kRxsBroken when the segment's chain does not hold it.
__device__ __forceinline__ uint64_t rxs_entry(uint64_t i, uint64_t E, uint64_t C, uint64_t prev, uint64_t len,
                                              const uint16_t *__restrict__ nodes) {
  if (C == kRxsBroken || prev == kRxsBroken) return kRxsBroken;
  if (E == prev) return 0;
  // the chain entered before the true entry: it holds it if it merged
  const uint64_t s0 = i * kRxsSeg;
  if (!(E < prev && prev < min(len, s0 + kRxsSeg))) return kRxsBroken;
  const uint16_t *nd = nodes + i * (kRxsSeg / 4);
  const uint32_t w = static_cast<uint32_t>((prev - s0) >> 2);
  uint64_t lo = 0, hi = C;
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (nd[m] < w) lo = m + 1; else hi = m;
  }
  return lo < C && nd[lo] == w ? lo : kRxsBroken;
}

// The walk's own verdict on segment i given its entry prev: its node index
// there, kRxsBroken when its chain does not hold prev; kRxsPassOver when no
// record starts in it (prev at or past its end).
constexpr uint64_t kRxsPassOver = ~1ull;
__device__ __forceinline__ uint64_t rxs_verdict(const uint64_t *__restrict__ seg, const uint16_t *__restrict__ nodes,
                                                uint64_t i, uint64_t nseg, uint64_t len, uint64_t prev) {
  if (prev != kRxsBroken && prev >= min(len, (i + 1) * kRxsSeg))
    return i == nseg - 1 && prev != len ? kRxsBroken : kRxsPassOver;
  const uint64_t *r = seg + i * kRxsSegWords;
  const uint64_t k = rxs_entry(i, r[0], r[2], prev, len, nodes);
  return k != kRxsBroken && (i != nseg - 1 || r[1] == len) ? k : kRxsBroken;
}

// One thread per segment: the true entry among the segment's nodes, against
// the previous segment's exit -- r[3] = its index, cnt[i] = the segment's
// records from it (for the scan); a segment where no record starts (the
// previous exit at or past its end) is passed over (0, 0).  A segment whose
// check fails clears the flag (the list ranking), except in a WHOLE walk
// (LONG), where it goes to rxs_fix's list -- a guess that missed there is
// expected: a look-back inside a long record's payload has no true chain to
// follow -- and so does a segment whose exit passes over a whole segment
// (the segments after it were passed over on its word).
template <bool LONG = false>
__device__ __forceinline__ void rxs_check_body(uint64_t *__restrict__ seg, const uint16_t *__restrict__ nodes,
                                               uint64_t nseg, uint64_t len, unsigned long long *__restrict__ cnt,
                                               uint32_t *__restrict__ flag, uint64_t *__restrict__ list,
                                               unsigned long long *nl) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nseg) return;
  uint64_t *r = seg + i * kRxsSegWords;
  const uint64_t prev = i == 0 ? 0 : seg[(i - 1) * kRxsSegWords + 1];
  const uint64_t k = rxs_verdict(seg, nodes, i, nseg, len, prev);
  const bool far = LONG && r[1] != kRxsBroken && r[1] >= (i + 2) * kRxsSeg;
  if (LONG && (far || k == kRxsBroken)) {
    list[atomicAdd(nl, 1ull)] = i;
    return;
  }
  if (k == kRxsPassOver) {  // no record starts in the segment
    r[3] = 0;
    cnt[i] = 0;
    return;
  }
  const bool ok = k != kRxsBroken;
  r[3] = ok ? k : 0;
  cnt[i] = ok ? r[2] - k : 0;
  if (!ok) *flag = 0u;
}

// rxs_fix (WHOLE walks): one wave, the listed segments in stream order, each
// from its true entry: a segment the entry passes over is passed over (no
// record starts there), one whose own walk holds the entry keeps its nodes,
// and any other is walked again by the wave from it (nodes, count, exit);
// when the exit differs from the one its own walk found -- which the next
// segment was checked against -- the next segment follows.  The entry of
// the first segment of such a run is the exit of a segment whose check held,
// so every entry is the true chain's (by induction from byte 0) and the
// index stays exact.  Each segment it decides gets r[3] and cnt as
// rxs_check's; a chain that does not parse, or a last segment that does not
// end at the stream's end, clears the flag, and so do more than kRxsFixCap
// listed segments (the list ranking).
constexpr uint32_t kRxsFixBits = 1u << 18;  // segments the fix's LDS bitmap covers (1.8 GB of stream)
constexpr uint64_t kRxsFixCap = 4096;       // listed segments it takes at most
template <class P>
__device__ __forceinline__ void rxs_fix_body(const P &parser, const uint8_t *__restrict__ s, uint64_t len,
                                             uint32_t maxlen, uint64_t *__restrict__ seg, uint64_t nseg,
                                             uint16_t *__restrict__ nodes, const uint64_t *__restrict__ list,
                                             const unsigned long long *nl, uint32_t *__restrict__ flag,
                                             unsigned long long *__restrict__ cnt) {
  __shared__ uint32_t bits[kRxsFixBits / 32];
  __shared__ __attribute__((aligned(16))) uint32_t blk[kRxsLongBlk / 4];
  extern __shared__ __attribute__((aligned(16))) uint32_t rx_smem[];
  const uint32_t lane = threadIdx.x;
  const uint64_t c = *nl;
  if (c == 0) return;
  if (nseg > kRxsFixBits || c > kRxsFixCap) {  // (the list ranking)
    if (lane == 0) *flag = 0u;
    return;
  }
  const uint32_t nw = static_cast<uint32_t>((nseg + 31) / 32);
  for (uint32_t j = lane; j < nw; j += 64u) bits[j] = 0u;
  wave_sync();
  for (uint64_t j = lane; j < c; j += 64u) {
    const uint64_t k = list[j];
    atomicOr(&bits[k >> 5], 1u << (k & 31u));
  }
  wave_sync();
  parser.init(rx_smem);
  const rx_blk rd{s, len, blk, 0};
  uint64_t cover = 0;  // segments below it are decided
  for (uint32_t j0 = 0; j0 < nw; j0 += 64u) {
    const uint32_t mine = j0 + lane < nw ? bits[j0 + lane] : 0u;
    uint64_t any = __ballot(mine != 0u);
    while (any) {
      const uint32_t l = __builtin_ctzll(any);
      any &= any - 1;
      uint32_t word = __shfl(mine, l, 64);
      while (word) {
        uint64_t i = 32ull * (j0 + l) + __builtin_ctz(word);
        word &= word - 1;
        if (i < cover) continue;  // decided by an earlier run
        // the run from i: its entry is the exit of segment i - 1, whose own
        // check held (it is not listed, or a run ended there)
        uint64_t x = i == 0 ? 0 : seg[(i - 1) * kRxsSegWords + 1];
        for (;;) {
          uint64_t *r = seg + i * kRxsSegWords;
          const uint64_t own = r[1];
          const uint64_t s0 = i * kRxsSeg, s1 = min(len, s0 + kRxsSeg);
          uint64_t q = x;
          bool ok = true;
          const uint64_t v = rxs_verdict(seg, nodes, i, nseg, len, x);
          if (v == kRxsPassOver) {  // passed over
            if (lane == 0) {
              r[3] = 0;
              cnt[i] = 0;
            }
          } else if (v != kRxsBroken) {  // its own walk holds from x
            q = own;
            if (lane == 0) {
              r[3] = v;
              cnt[i] = r[2] - v;
            }
          } else {  // walked again from x: its records' nodes, count and exit
            uint64_t m = 0;
            if (x != kRxsBroken) {
              rd.load(q);
              while (q < s1) {
                if (lane == 0) nodes[i * (kRxsSeg / 4) + m] = static_cast<uint16_t>((q - s0) >> 2);
                ++m;
                const uint32_t L = parser.template rlen_rd<rx_blk, uint64_t>(rx_smem, rd, len, q, maxlen);
                if (L >= RX_OUT) {
                  ok = false;
                  break;
                }
                q += L;
              }
            } else {
              ok = false;
            }
            if (i == nseg - 1 && q != len) ok = false;
            if (lane == 0) {
              r[0] = x;
              r[1] = ok ? q : kRxsBroken;
              r[2] = ok ? m : kRxsBroken;
              r[3] = 0;
              cnt[i] = ok ? m : 0;
              if (!ok) *flag = 0u;
            }
          }
          cover = i + 1;
          if (!ok || i + 1 >= nseg) break;
          // the next segment was checked against the exit its walk found:
          // it follows when that is not the true one, or when the true one
          // passes over it
          if (q == own && q < (i + 2) * kRxsSeg) break;
          ++i;
          x = q;
        }
      }
    }
  }
}

// One wave per segment (four to a 256-lane workgroup: a 64-lane workgroup
// per segment left rpc's 36K-segment emit at 12.8 us, dispatch-bound): its
// records' offsets, when every check held (the flag) and the chain holds
// exactly n records (EXACT: records of xdrg_index_records) or at most n
// (messages of xdrg_index_msgs, n = the capacity) -- the scan's total; the
// first wave also writes offsets[total], the count and the final flag.
constexpr uint32_t kRxsEmitWaves = 4;
template <bool EXACT>
__device__ __forceinline__ void rxs_emit_body(const uint64_t *__restrict__ seg, const uint16_t *__restrict__ nodes,
                                              const unsigned long long *__restrict__ base,
                                              const xdrg_status *__restrict__ tot, uint64_t len, uint64_t n,
                                              uint64_t *__restrict__ offsets, uint64_t *__restrict__ count,
                                              uint32_t *__restrict__ flag, uint64_t nseg, uint32_t *hflag,
                                              const unsigned long long *__restrict__ cnt) {
  const uint64_t t = tot->total_bytes;
  const bool all = *flag == 1u && (EXACT ? t == n : t <= n);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *flag = all ? 1u : 0u;
    if (hflag) *hflag = all ? 1u : 0u;  // the verdict the host waits for (mapped host memory)
    if (all) {
      offsets[t] = len;
      *count = t;
    }
  }
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kRxsEmitWaves + (threadIdx.x >> 6);
  if (!all || i >= nseg) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t *r = seg + i * kRxsSegWords;
  const uint64_t k = r[3], c = cnt[i], b0 = base[i], s0 = i * kRxsSeg;
  const uint16_t *in = nodes + i * (kRxsSeg / 4) + k;
  for (uint32_t j = lane; j < c; j += 64u) offsets[b0 + j] = s0 + 4ull * in[j];
}


}  // namespace dev
}  // namespace xdrg
