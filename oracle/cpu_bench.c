/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  The "port" CPU baseline of bench.py:
 * the C restatement of xdr_put / xdr_get (xdr_oracle.c, pinned to the real
 * reference by tests/test_oracle.py) run on every host core, the way the
 * reference's callers would batch it.  Never part of the product path.
 *
 *   xdro_bench   one pthread per requested core over contiguous record
 *                slices (SURVEY.md §8(d) CPU reference timing):
 *                  encode  = one xdr_put stream over the slice
 *                        (xdr_to_opaque(r_a, ..., r_b-1), marshal.h:264-272)
 *                  decode  = one xdr_get stream over the slice
 *                        (xdr_from_opaque, marshal.h:299-306)
 *                  to_opaque = per-record allocating xdr_to_opaque (malloc
 *                        of xdr_size bytes, encode, copy out, free), as RPC
 *                        callers do (srpc.h:58 via xdr_to_msg)
 *                Output buffers are pre-faulted by an untimed pass; best and
 *                median of `reps`.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/xdrgpu.h"

int xdro_encode(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                const uint8_t *native, uint64_t n, const uint8_t *heap, uint64_t heap_len,
                uint8_t *out, uint64_t cap, uint64_t *offsets, uint32_t stack_limit,
                uint64_t *erec, uint32_t *eop, uint64_t *total);
int xdro_decode(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                const uint8_t *xdr, uint64_t len, const uint64_t *offsets, uint64_t n,
                uint8_t *native, uint8_t *heap_out, uint32_t stack_limit, uint64_t *erec,
                uint32_t *eop);
int xdro_sizes(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
               const uint8_t *native, uint64_t n, const uint8_t *heap, uint64_t heap_len,
               uint32_t *sizes, uint64_t *erec, uint32_t *eop);
uint64_t xdro_decode_heap_size(const xdrg_op *ops, uint32_t nops, uint64_t len);

typedef struct {
  const xdrg_op *ops;
  uint32_t nops;
  const uint32_t *table;
  uint32_t stride;
  const uint8_t *native;
  const uint8_t *heap;
  uint64_t heap_len;
  uint8_t *out, *back;
  uint8_t *hout;       /* the thread's decoded heap (element arrays), or NULL */
  const uint64_t *off; /* record offsets, n + 1 */
  const uint32_t *sizes;
  uint64_t a, b;       /* the thread's record slice */
  int mode;            /* 0 encode, 1 decode, 2 per-record to_opaque */
  int rc;
} job_t;

static void *run_job(void *arg) {
  job_t *j = (job_t *)arg;
  uint64_t erec = 0, total = 0;
  uint32_t eop = 0;
  const uint64_t a = j->a, b = j->b;
  if (a >= b) return NULL;
  uint8_t *dst = j->out + j->off[a];
  const uint64_t len = j->off[b] - j->off[a];
  if (j->mode == 0) {
    j->rc = xdro_encode(j->ops, j->nops, j->table, j->stride, j->native + a * j->stride, b - a,
                        j->heap, j->heap_len, dst, len, NULL, 0xffffffffu, &erec, &eop, &total);
  } else if (j->mode == 1) {
    j->rc = xdro_decode(j->ops, j->nops, j->table, j->stride, dst, len, NULL, b - a,
                        j->back + a * j->stride, j->hout, 0xffffffffu, &erec, &eop);
  } else {
    for (uint64_t r = a; r < b && !j->rc; ++r) {
      const uint32_t sz = j->sizes[r];
      uint8_t *m = (uint8_t *)malloc(sz ? sz : 4);
      j->rc = xdro_encode(j->ops, j->nops, j->table, j->stride, j->native + r * j->stride, 1,
                          j->heap, j->heap_len, m, sz, NULL, 0xffffffffu, &erec, &eop, &total);
      memcpy(j->out + j->off[r], m, sz);
      free(m);
    }
  }
  return NULL;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int cmp_d(const void *x, const void *y) {
  const double a = *(const double *)x, b = *(const double *)y;
  return a < b ? -1 : a > b;
}

/* Runs `mode` over n records on `threads` threads; returns seconds or < 0. */
static double run_all(job_t *proto, uint64_t n, uint32_t threads, int mode, pthread_t *th, job_t *jobs,
                      uint8_t **houts) {
  const double t0 = now_s();
  for (uint32_t t = 0; t < threads; ++t) {
    jobs[t] = *proto;
    jobs[t].mode = mode;
    jobs[t].a = n * t / threads;
    jobs[t].b = n * (t + 1) / threads;
    jobs[t].rc = 0;
    jobs[t].hout = houts[t];
    if (pthread_create(&th[t], NULL, run_job, &jobs[t])) return -1.0;
  }
  int rc = 0;
  for (uint32_t t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    rc |= jobs[t].rc;
  }
  const double dt = now_s() - t0;
  return rc ? -2.0 : dt;
}

/*
 * out:  caller buffer of at least xdr_size(batch) bytes (receives the
 *       encoded stream, so the caller can check it against the reference's
 *       hash); back: n * stride bytes (decoded records).
 * res[0..7] = encode best, encode median, decode best, decode median,
 *             to_opaque best, to_opaque median, xdr bytes, threads.
 * A plan with containers decodes each slice's element arrays into a heap
 * of the thread's own (xdro_decode's heap_out: the slice's stream copy,
 * then the arrays), allocated and pre-faulted before the timed runs.
 * Returns 0, or a negative value (thread or marshal failure).
 */
int xdro_bench(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
               const uint8_t *native, uint64_t n, const uint8_t *heap, uint64_t heap_len,
               uint8_t *out, uint64_t out_cap, uint8_t *back, uint32_t threads, uint32_t reps,
               double *res) {
  if (!threads || !reps || reps > 64 || !n) return -1;
  uint32_t *sizes = (uint32_t *)malloc(n * sizeof(uint32_t));
  uint64_t *off = (uint64_t *)malloc((n + 1) * sizeof(uint64_t));
  pthread_t *th = (pthread_t *)malloc(threads * sizeof(pthread_t));
  job_t *jobs = (job_t *)malloc(threads * sizeof(job_t));
  uint8_t **houts = (uint8_t **)calloc(threads, sizeof(uint8_t *));
  int rc = 0;
  if (!sizes || !off || !th || !jobs || !houts) { rc = -3; goto done; }
  {
    uint64_t erec = 0;
    uint32_t eop = 0;
    if (xdro_sizes(ops, nops, table, stride, native, n, heap, heap_len, sizes, &erec, &eop)) { rc = -4; goto done; }
    off[0] = 0;
    for (uint64_t r = 0; r < n; ++r) off[r + 1] = off[r] + sizes[r];
    if (off[n] > out_cap) { rc = -5; goto done; }
    for (uint32_t t = 0; t < threads; ++t) {
      const uint64_t len = off[n * (t + 1) / threads] - off[n * t / threads];
      const uint64_t hb = xdro_decode_heap_size(ops, nops, len);
      if (hb > len && !(houts[t] = (uint8_t *)calloc(hb ? hb : 1, 1))) { rc = -3; goto done; }
    }
    job_t proto = {ops, nops, table, stride, native, heap, heap_len, out, back, NULL, off, sizes, 0, 0, 0, 0};
    double te[64], td[64], tp[64];
    if (run_all(&proto, n, threads, 0, th, jobs, houts) < 0 || run_all(&proto, n, threads, 1, th, jobs, houts) < 0 ||
        run_all(&proto, n, threads, 2, th, jobs, houts) < 0) { rc = -6; goto done; }
    for (uint32_t i = 0; i < reps; ++i) {
      te[i] = run_all(&proto, n, threads, 0, th, jobs, houts);
      td[i] = run_all(&proto, n, threads, 1, th, jobs, houts);
      tp[i] = run_all(&proto, n, threads, 2, th, jobs, houts);
      if (te[i] < 0 || td[i] < 0 || tp[i] < 0) { rc = -6; goto done; }
    }
    qsort(te, reps, sizeof(double), cmp_d);
    qsort(td, reps, sizeof(double), cmp_d);
    qsort(tp, reps, sizeof(double), cmp_d);
    res[0] = te[0]; res[1] = te[reps / 2];
    res[2] = td[0]; res[3] = td[reps / 2];
    res[4] = tp[0]; res[5] = tp[reps / 2];
    res[6] = (double)off[n];
    res[7] = (double)threads;
  }
done:
  free(sizes);
  free(off);
  free(th);
  free(jobs);
  if (houts)
    for (uint32_t t = 0; t < threads; ++t) free(houts[t]);
  free(houts);
  return rc;
}
