/* Tuning tool (not product, not a test): simulates the speculative record
 * index on the CPU over a real stream, to measure how often a segment's
 * guessed chain misses the true one and how many lane rounds the
 * in-segment fixpoint takes.  Reuses the oracle's record parse (rx_walk).
 *   gcc -O2 -shared -fPIC -o /tmp/rx_spec_sim.so tools/tune/rx_spec_sim.c
 */
#include "../../oracle/xdr_oracle.c"

/* length of the record at p (0 = does not parse) */
static uint64_t rlen(const plan_t *P, const uint8_t *s, uint64_t len, uint64_t p, uint32_t maxlen) {
  const int capped = p + maxlen < len;
  rxctx c = {P, s, capped ? p + maxlen : len, capped ? RX_LONG : RX_BAD};
  uint64_t q = p;
  if (p >= len) return 0;
  if (rx_walk(&c, &q, 0, 0)) return 0;
  return q - p;
}

/* chain from p until >= end: returns exit (or ~0 when a record fails) */
static uint64_t walk(const plan_t *P, const uint8_t *s, uint64_t len, uint64_t p, uint64_t end,
                     uint32_t maxlen, uint64_t *steps) {
  while (p < end) {
    uint64_t L = rlen(P, s, len, p, maxlen);
    ++*steps;
    if (!L) return ~0ull;
    p += L;
  }
  return p;
}
static int on_chain(const plan_t *P, const uint8_t *s, uint64_t len, uint64_t from, uint64_t target,
                    uint32_t maxlen) {
  uint64_t p = from, st = 0;
  while (p < target) {
    uint64_t L = rlen(P, s, len, p, maxlen);
    if (!L) return 0;
    p += L;
  }
  (void)st;
  return p == target;
}

typedef struct {
  uint64_t segs, seg_fail, lanes, lanes_noguess, lanes_sync0, guess_tries, walk_steps, max_rounds, sum_rounds;
} stats_t;

void sim(const xdrg_op *ops, uint32_t nops, const uint32_t *table, const uint8_t *s, uint64_t len,
         uint32_t maxlen, uint32_t SEG, uint32_t SUB, uint32_t back, stats_t *st) {
  plan_t P = {ops, nops, table, 0, NULL};
  memset(st, 0, sizeof *st);
  const uint32_t NL = SEG / SUB;
  uint64_t *g = malloc(NL * 8), *e = malloc(NL * 8), *ent = malloc(NL * 8);
  /* true chain exits per segment */
  uint64_t truep = 0;
  for (uint64_t s0 = 0; s0 < len; s0 += SEG) {
    const uint64_t s1 = s0 + SEG < len ? s0 + SEG : len;
    st->segs++;
    /* lane guesses */
    for (uint32_t j = 0; j < NL; ++j) {
      uint64_t a = s0 + (uint64_t)j * SUB, b = a + SUB < s1 ? a + SUB : s1;
      g[j] = ~0ull; e[j] = ~0ull;
      if (a >= s1) continue;
      st->lanes++;
      uint64_t a0 = (j == 0 && a >= back) ? a - back : a;  /* lane 0 may start earlier */
      for (uint64_t p = a0; p < b; p += 4) {
        st->guess_tries++;
        uint64_t x = walk(&P, s, len, p, b, maxlen, &st->walk_steps);
        if (x != ~0ull) { g[j] = p; e[j] = x; break; }
      }
      if (g[j] == ~0ull) st->lanes_noguess++;
    }
    /* fixpoint over lanes, rooted at lane 0's guess (segment guess) */
    uint64_t rounds = 0;
    for (uint32_t j = 0; j < NL; ++j) ent[j] = ~0ull;
    /* lane j synced if its entry (exit of j-1) is on its guess chain */
    uint64_t prev = g[0] == ~0ull ? s0 : g[0];
    uint64_t segexit = prev;
    for (uint32_t j = 0; j < NL; ++j) {
      uint64_t a = s0 + (uint64_t)j * SUB, b = a + SUB < s1 ? a + SUB : s1;
      if (a >= s1) break;
      if (j == 0) { segexit = e[0] == ~0ull ? b : e[0]; continue; }
      if (segexit >= b) continue;  /* passed through */
      if (g[j] != ~0ull && g[j] <= segexit && on_chain(&P, s, len, g[j], segexit, maxlen)) {
        st->lanes_sync0++;
        segexit = e[j];
      } else {
        ++rounds;
        segexit = walk(&P, s, len, segexit, b, maxlen, &st->walk_steps);
        if (segexit == ~0ull) break;
      }
    }
    st->sum_rounds += rounds;
    if (rounds > st->max_rounds) st->max_rounds = rounds;
    /* segment check: true entry on the segment's guessed chain */
    uint64_t G = g[0];
    int ok = (G != ~0ull) && G <= truep && on_chain(&P, s, len, G, truep, maxlen);
    if (truep >= s1) ok = 1;  /* passed through by a long record (handled apart) */
    if (!ok) st->seg_fail++;
    /* advance the true chain past this segment */
    if (truep < s1) {
      uint64_t x = walk(&P, s, len, truep, s1, maxlen, &st->walk_steps);
      if (x == ~0ull) break;
      truep = x;
    }
  }
  free(g); free(e); free(ent);
}

/* Wave-faithful model of rxs_walk_body (index_kernels.h): per wave, the
 * record parses each lane runs in each phase, and the SIMT cost (the
 * largest count over the lanes, per phase).  first_ok is approximated by
 * "rlen does not fail at the first checked word" (counted apart). */
typedef struct {
  uint64_t waves, parses_guess, parses_fix, parses_nodes, simt_guess, simt_fix, simt_nodes, fix_rounds, cands,
      simt_cands;
} wstats_t;

void sim_wave(const xdrg_op *ops, uint32_t nops, const uint32_t *table, const uint8_t *s, uint64_t len,
              uint32_t maxlen, uint32_t SUB, uint32_t BACKL, uint32_t FD, wstats_t *w) {
  plan_t P = {ops, nops, table, 0, NULL};
  memset(w, 0, sizeof *w);
  const uint32_t SEG = (64 - BACKL) * SUB;
  for (uint64_t s0 = 0; s0 < len; s0 += SEG) {
    const uint64_t s1 = s0 + SEG < len ? s0 + SEG : len;
    const int first = s0 == 0;
    const uint32_t root = first ? BACKL : 0;
    uint64_t g[64], e[64], g0[64], e0[64], pin[64];
    uint64_t pg[64] = {0}, pf[64] = {0}, pn[64] = {0}, cn[64] = {0};
    w->waves++;
    for (uint32_t j = 0; j < 64; ++j) {
      g[j] = e[j] = ~0ull - 1;
      int64_t a = (int64_t)s0 + (int64_t)SUB * j - (int64_t)BACKL * SUB;
      uint64_t b = (uint64_t)a + SUB < s1 ? (uint64_t)a + SUB : s1;
      int act = j >= root && a >= 0 && (uint64_t)a < s1;
      if (!act) continue;
      if (first && j == root) {
        uint64_t st = 0;
        g[j] = 0; e[j] = walk(&P, s, len, 0, b, maxlen, &st); pg[j] += st;
      } else {
        for (uint64_t p = a; p < b; p += 4) {
          /* candidate = the parse gets past its first checked word (a walk
           * capped right after it does not fail on it) */
          if (FD != ~0u) {
            rxctx c = {&P, s, p + FD + 4 < len ? p + FD + 4 : len, RX_LONG};
            uint64_t q = p;
            if (rx_walk(&c, &q, 0, 0) == RX_BAD) continue;
          }
          uint64_t st = 0;
          uint64_t q = walk(&P, s, len, p, b, maxlen, &st);
          pg[j] += st; cn[j]++;
          if (q != ~0ull) { g[j] = p; e[j] = q; break; }
        }
        if (g[j] == ~0ull - 1 && (j == root || j < BACKL)) e[j] = ~0ull;
      }
    }
    for (uint32_t j = 0; j < 64; ++j) { g0[j] = g[j]; e0[j] = e[j]; pin[j] = g[j]; }
    for (int it = 0; it < 64; ++it) {
      uint64_t pe[64];
      int ch = 0;
      for (uint32_t j = 0; j < 64; ++j) pe[j] = j ? e[j - 1] : 0;
      for (uint32_t j = 0; j < 64; ++j) {
        int64_t a = (int64_t)s0 + (int64_t)SUB * j - (int64_t)BACKL * SUB;
        uint64_t b = (uint64_t)a + SUB < s1 ? (uint64_t)a + SUB : s1;
        int act = j >= root && a >= 0 && (uint64_t)a < s1;
        if (j > root && pe[j] != ~0ull - 1 && pe[j] != pin[j]) {
          ch = 1;
          pin[j] = g[j] = pe[j];
          if (pe[j] == ~0ull || !act || pe[j] >= b) e[j] = pe[j];
          else { uint64_t st = 0; e[j] = walk(&P, s, len, pe[j], b, maxlen, &st); pf[j] += st; }
          if (e[j] == ~0ull && j < BACKL) { g[j] = g0[j]; e[j] = e0[j]; }
        }
      }
      if (!ch) break;
      w->fix_rounds++;
    }
    uint64_t mg = 0, mf = 0, mn = 0, mc = 0;
    for (uint32_t j = 0; j < 64; ++j) {
      int64_t a = (int64_t)s0 + (int64_t)SUB * j - (int64_t)BACKL * SUB;
      uint64_t b = (uint64_t)a + SUB < s1 ? (uint64_t)a + SUB : s1;
      if (j >= BACKL && a >= 0 && (uint64_t)a < s1 && e[j] != ~0ull)
        for (uint64_t q = g[j]; q < b;) { q += rlen(&P, s, len, q, maxlen); pn[j] += 2; }
      w->parses_guess += pg[j]; w->parses_fix += pf[j]; w->parses_nodes += pn[j]; w->cands += cn[j];
      if (pg[j] > mg) mg = pg[j];
      if (pf[j] > mf) mf = pf[j];
      if (pn[j] > mn) mn = pn[j];
      if (cn[j] > mc) mc = cn[j];
    }
    w->simt_guess += mg; w->simt_fix += mf; w->simt_nodes += mn; w->simt_cands += mc;
  }
}
