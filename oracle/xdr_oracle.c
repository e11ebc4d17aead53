/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Imported by tests/, by
 * __graft_entry__.smoke() as the checker, and by bench.py's cpu_baseline leg
 * (as the "port" CPU baseline when the reference build is absent).  Never
 * part of the product path.
 *
 * A scalar CPU restatement of xdrpp's marshal hot path, driven by the same
 * flat plan (xdrg_op[]) the GPU kernels execute.  Every step follows the
 * reference archive one field at a time:
 *
 *   check(n) before every read/write     xdrpp/marshal.h:104-108 (put),
 *                                        :166-170 (get)
 *   put32/put64 = swap32 per word, high  xdrpp/marshal.h:65-80,
 *   word first for 64-bit                xdrpp/endian.h:56-68
 *   bytes: length word if variable,      xdrpp/marshal.h:118-127 (put),
 *   memcpy, zero pad to 4 / verify pad   :185-196 (get), marshal.cc:43-72
 *   bool decodes nonzero as true         xdrpp/types.h:335-349
 *   opt-in enum validation               xdrpp/types.h:157-173
 *   union: discriminant, then arm;       xdrc/gen_hh.cc:639-673, :472-487
 *   unknown -> bad discriminant
 *   stack budget per class level         xdrpp/marshal.h:129-136, :198-205
 *   misaligned end / trailing bytes      xdrpp/marshal.h:152-162, :207-210
 *
 * Parity of this restatement is pinned by tests/test_oracle.py against the
 * golden fixtures that oracle/ref_golden (the real reference, compiled from
 * /root/reference) produced.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/xdrgpu.h"

static inline uint32_t bswap32(uint32_t v) {
  return v << 24 | (v & 0xff00) << 8 | (v >> 8 & 0xff00) | v >> 24;
}
static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static inline void wr64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline uint64_t pad4(uint64_t n) { return (n + 3) & ~(uint64_t)3; }

typedef struct {
  const xdrg_op *ops;
  uint32_t nops;
  const uint32_t *table;
  uint32_t stride;
  const uint64_t *minw; /* decode: least wire bytes from each pc to its END */
} plan_t;

/* Find the target pc of a union discriminant, or -1. */
static int64_t union_target(const plan_t *P, const xdrg_op *op, uint32_t disc) {
  const uint32_t *ct = P->table + op->arg2;
  for (uint32_t i = 0; i < op->arg3; ++i)
    if (ct[2 * i] == disc) return ct[2 * i + 1];
  if (op->flags & XDRG_F_DEFAULT) return op->arg4;
  return -1;
}
static int enum_ok(const plan_t *P, const xdrg_op *op, uint32_t v) {
  if (!(op->flags & XDRG_F_VALIDATE)) return 1;
  const uint32_t *t = P->table + op->arg0;
  for (uint32_t i = 0; i < op->arg1; ++i)
    if (t[i] == v) return 1;
  return 0;
}

/* Plan regions.  The record's ops end with END; element subroutines
 * (XDRG_F_SUB VECTOR ops, arg4 = entry pc) follow, each ending with END.
 * A subroutine walks one element: field offsets relative to the element,
 * depths relative to the VECTOR op that entered it (dbase).  The reference
 * recurses on its C++ stack (types.h:374-392, marshal.h:129-136); so does
 * this restatement, with no bound on the nesting but marshaling_stack_limit
 * (the device's XDRG_MAX_FRAMES lies past the depth at which the
 * reference's own recursion overflows its call stack, and past this one's).
 *
 * Native objects are read through obj_t: the record (stride bytes) or an
 * element in the heap; bytes at or past the end read as 0, as the kernels'
 * clamped loads do. */
typedef struct {
  const uint8_t *base;
  uint64_t len;
  uint64_t off;
} obj_t;
static inline uint8_t o8(obj_t o, uint64_t k) { return o.off + k < o.len ? o.base[o.off + k] : 0; }
static inline uint32_t o32(obj_t o, uint64_t k) {
  if (o.off + k + 4 <= o.len) return rd32(o.base + o.off + k);
  uint8_t b[4];
  for (int i = 0; i < 4; ++i) b[i] = o8(o, k + (uint64_t)i);
  return rd32(b);
}
/* n bytes of o from k into w (bytes past the end read 0) */
static inline void obytes(obj_t o, uint64_t k, uint8_t *w, uint64_t n) {
  if (o.off + k + n <= o.len) { memcpy(w, o.base + o.off + k, n); return; }
  for (uint64_t i = 0; i < n; ++i) w[i] = o8(o, k + i);
}
static inline uint64_t o64(obj_t o, uint64_t k) { return o32(o, k) | (uint64_t)o32(o, k + 4) << 32; }

/* Fixed-size elements of a VECTOR op without F_SUB: ops [pc+1, pc+1+arg2). */
static uint32_t elem_wire(const xdrg_op *e) {
  return e->kind == XDRG_OP_U64 ? 8u : e->kind == XDRG_OP_OPAQUE ? pad4(e->arg0) : 4u;
}
static uint32_t vec_wire(const plan_t *P, uint32_t pc) {
  uint32_t w = 0;
  for (uint32_t k = 1; k <= P->ops[pc].arg2; ++k) w += elem_wire(&P->ops[pc + k]);
  return w;
}
/* Decoded element arrays of record r come from [align16(len) + F * off[r],
 * align16(len) + F * off[r+1]) for recursive plans (element subroutines
 * that can nest past XDRG_SUB_FRAMES), packed per group of 64 records
 * otherwise (rec_ebytes below).  Fixed elements:
 * F = 1 + the largest native/wire size ratio of an element type (+ 2 when
 * packed).  Subroutine elements: distinct elements start at distinct wire
 * words, so stride/4 per wire byte, plus 2 for the 8-byte alignment of each
 * array (xdrpp_amd/csrc/plan.cpp). */
/* Least wire bytes of the walk from each pc to its region's END (unions:
 * the cheapest arm; containers: empty), as plan.cpp computes them: an
 * element subroutine consumes at least minw[body] bytes per element. */
static uint64_t *min_wires(const xdrg_op *ops, uint32_t nops, const uint32_t *table) {
  uint64_t *m = (uint64_t *)calloc((size_t)nops + 1, sizeof *m);
  if (!m) abort();
  for (uint32_t i = nops; i-- > 0;) {
    const xdrg_op *op = &ops[i];
    uint64_t v = 0;
    switch (op->kind) {
    case XDRG_OP_END: v = 0; break;
    case XDRG_OP_JUMP: v = m[op->arg0]; break;
    case XDRG_OP_VECTOR: v = m[i + 1 + op->arg2] + 4; break;
    case XDRG_OP_UNION: {
      int any = 0;
      for (uint32_t c = 0; c < op->arg3; ++c) {
        const uint64_t t = m[table[op->arg2 + 2 * c + 1]];
        if (!any || t < v) v = t;
        any = 1;
      }
      if (op->flags & XDRG_F_DEFAULT) {
        const uint64_t t = m[op->arg4];
        if (!any || t < v) v = t;
      }
      v += 4;
      break;
    }
    case XDRG_OP_U64: v = m[i + 1] + 8; break;
    case XDRG_OP_OPAQUE: v = m[i + 1] + pad4(op->arg0); break;
    default: v = m[i + 1] + 4; break;
    }
    m[i] = v;
  }
  return m;
}

/* Element-subroutine frames a walk entering the region at `start` can
 * open below it (UINT32_MAX: the region can enter itself -- a recursive
 * type), as plan.cpp computes them; on[] marks the regions on the path. */
static uint32_t sub_frames(const plan_t *P, uint32_t start, uint8_t *on) {
  uint32_t f = 0;
  on[start] = 1;
  for (uint32_t pc = start; pc < P->nops && P->ops[pc].kind != XDRG_OP_END; ++pc) {
    const xdrg_op *op = &P->ops[pc];
    if (op->kind != XDRG_OP_VECTOR || !(op->flags & XDRG_F_SUB)) continue;
    uint32_t g = on[op->arg4] ? UINT32_MAX : sub_frames(P, op->arg4, on);
    g = g == UINT32_MAX ? UINT32_MAX : g + 1;
    if (g > f) f = g;
  }
  on[start] = 0;
  return f;
}
/* Plans with containers whose walks never need the deep passes (at most
 * XDRG_SUB_FRAMES element frames, no recursive type) pack each group of 64
 * records' arrays back to back (below); their factor carries 2 more bytes
 * per wire byte for the 8-byte rounding of every array
 * (xdrpp_amd/csrc/plan.cpp).  Recursive plans keep per-record areas. */
static int packed_plan(const plan_t *P) {
  int vec = 0;
  for (uint32_t pc = 0; pc < P->nops; ++pc)
    if (P->ops[pc].kind == XDRG_OP_VECTOR) vec = 1;
  if (!vec) return 0;
  uint8_t *on = (uint8_t *)calloc((size_t)P->nops + 1, 1);
  if (!on) abort();
  const uint32_t f = sub_frames(P, 0, on);
  free(on);
  return f <= XDRG_SUB_FRAMES;
}
static uint32_t heap_factor(const plan_t *P) {
  uint32_t f = 0;
  for (uint32_t pc = 0; pc < P->nops; ++pc)
    if (P->ops[pc].kind == XDRG_OP_VECTOR) {
      const xdrg_op *op = &P->ops[pc];
      uint32_t g;
      if (op->flags & XDRG_F_SUB) {
        g = (op->arg1 + 3) / 4 + 2;
      } else {
        uint32_t we = vec_wire(P, pc);
        g = (op->arg1 + we - 1) / we + 1;
      }
      if (g > f) f = g;
    }
  return f && packed_plan(P) ? f + 2 : f;
}

/* Packed element areas.  Records go in groups of 64 (records 64g ..
 * 64g+63 of the batch); group g's arrays start at align8(ebase + F *
 * off[64g]) and follow each other record by record, each array rounded up
 * to 8 bytes.  Record r's share is E(r): a walk of its structure (lengths,
 * counts, discriminants; no value checks) adding align8(min(cnt, rem /
 * wire + 1) * stride) per container, rem = the record's bytes after the
 * count, stopping where the structure stops parsing -- what the decode's
 * area check (elem_area_ok) needs, so valid records always fit; an element
 * subroutine's array counts align8(cnt * stride) when the bytes left can
 * hold its count, then its elements' own arrays -- capped at
 * align8-down(F * (b - a) - 8) so that no group outgrows its F-sized area.
 * The device kernels compute the same E(r) before their walks and place
 * the group's records by a wave scan (xdrpp_amd/csrc: dec_ebytes,
 * codegen.cpp ebytes). */
/* From pc to its region's END; *pp advanced.  Returns 0 where the
 * structure stops parsing (E holds the arrays up to there). */
static int ebytes_ops(const plan_t *P, const uint8_t *s, uint64_t *pp, uint64_t b, uint32_t pc, uint64_t *E) {
  uint64_t p = *pp;
  for (;;) {
    const xdrg_op *op = &P->ops[pc];
    switch (op->kind) {
    case XDRG_OP_END: *pp = p; return 1;
    case XDRG_OP_JUMP: pc = op->arg0; continue;
    case XDRG_OP_U64: if (b - p < 8) return 0; p += 8; ++pc; continue;
    case XDRG_OP_OPAQUE: if (b - p < op->arg0) return 0; p += pad4(op->arg0); ++pc; continue;
    case XDRG_OP_U32: case XDRG_OP_BOOL: case XDRG_OP_ENUM: if (b - p < 4) return 0; p += 4; ++pc; continue;
    default: break;
    }
    if (b - p < 4) return 0;
    const uint32_t v = bswap32(rd32(s + p));
    p += 4;
    switch (op->kind) {
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
      if (v > op->arg0 || b - p < v) return 0;
      p += pad4(v);
      ++pc;
      break;
    case XDRG_OP_UNION: {
      const int64_t t = union_target(P, op, v);
      if (t < 0) return 0;
      pc = (uint32_t)t;
      break;
    }
    case XDRG_OP_VECTOR: {
      if (v > op->arg0) return 0;
      const uint64_t rem = b - p;
      if (op->flags & XDRG_F_SUB) {  /* every element consumes at least minw[body] bytes */
        if ((uint64_t)v * P->minw[op->arg4] > rem) return 0;
        *E += ((uint64_t)v * op->arg1 + 7) & ~7ull;
        for (uint32_t i = 0; i < v; ++i)
          if (!ebytes_ops(P, s, &p, b, op->arg4, E)) return 0;
        ++pc;
        break;
      }
      const uint64_t w = vec_wire(P, pc);
      const uint64_t k = rem / w + 1 < v ? rem / w + 1 : v;
      *E += (k * op->arg1 + 7) & ~7ull;
      if (rem < (uint64_t)v * w) return 0;
      p += (uint64_t)v * w;
      pc += 1 + op->arg2;
      break;
    }
    default: ++pc; break;
    }
  }
}
static uint64_t rec_ebytes(const plan_t *P, const uint8_t *s, uint64_t p, uint64_t b) {
  uint64_t E = 0;
  (void)ebytes_ops(P, s, &p, b, 0, &E);
  return E;
}
static uint64_t ebudget(uint32_t F, uint64_t a, uint64_t b) {
  const uint64_t t = (uint64_t)F * (b - a);
  return t >= 8 ? (t - 8) & ~7ull : 0;
}
uint64_t xdro_decode_heap_size(const xdrg_op *ops, uint32_t nops, uint64_t len) {
  plan_t P = {ops, nops, NULL, 0, NULL};
  uint32_t f = heap_factor(&P);
  return f ? ((len + 15) & ~15ull) + (uint64_t)f * len : len;
}

/* ------------------------------------------------------------------ size */
/* xdr_size (xdr_traits<T>::serial_size) of the object from pc to its END,
 * and the deepest class/container level entered (depth_checker,
 * xdrpp/depth_checker.h:10-79: a union and a container count their own
 * level, a non-empty xvector/pointer its element's).  A bad discriminant
 * sets c->err / c->eop. */
typedef struct {
  const plan_t *P;
  const uint8_t *heap;
  uint64_t heap_len;
  uint32_t err, eop, dmax;
} szctx;
static uint64_t size_ops(szctx *c, uint32_t pc, obj_t o, uint32_t dbase) {
  const plan_t *P = c->P;
  uint64_t s = 0;
  for (;;) {
    const xdrg_op *op = &P->ops[pc];
    if (op->kind == XDRG_OP_END) return s;
    if (op->kind == XDRG_OP_JUMP) { pc = op->arg0; continue; }
    if (dbase + op->depth > c->dmax) c->dmax = dbase + op->depth;
    switch (op->kind) {
    case XDRG_OP_U64: s += 8; ++pc; break;
    case XDRG_OP_OPAQUE: s += pad4(op->arg0); ++pc; break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: s += 4 + pad4(o32(o, op->noff + 8)); ++pc; break;
    case XDRG_OP_UNION: {
      int64_t t = union_target(P, op, o32(o, op->noff));
      if (t < 0) { c->err = XDRG_ERR_BAD_DISCRIMINANT; c->eop = pc; return 0; }
      s += 4;
      pc = (uint32_t)t;
      break;
    }
    case XDRG_OP_VECTOR: {
      const uint64_t eoff = o64(o, op->noff);
      const uint32_t cnt = o32(o, op->noff + 8);
      s += 4;
      if (!(op->flags & XDRG_F_SUB)) {
        s += (uint64_t)cnt * vec_wire(P, pc);
        if (cnt)
          for (uint32_t k = 1; k <= op->arg2; ++k)
            if (dbase + P->ops[pc + k].depth > c->dmax) c->dmax = dbase + P->ops[pc + k].depth;
        pc += 1 + op->arg2;
        break;
      }
      for (uint32_t i = 0; i < cnt; ++i) {
        obj_t e = {c->heap, c->heap_len, eoff + (uint64_t)i * op->arg1};
        s += size_ops(c, op->arg4, e, dbase + op->depth);
        if (c->err) return 0;
      }
      ++pc;
      break;
    }
    default: s += 4; ++pc; break;
    }
  }
}
static uint64_t rec_size(const plan_t *P, const uint8_t *nat, const uint8_t *heap, uint64_t heap_len,
                         uint32_t *err, uint32_t *eop) {
  szctx c = {P, heap, heap_len, 0, 0, 0};
  obj_t o = {nat, P->stride, 0};
  uint64_t s = size_ops(&c, 0, o, 0);
  *err = c.err;
  *eop = c.eop;
  return s;
}

/* ---------------------------------------------------------------- encode */
/* xdr_generic_put of the object from pc to its END: check(n) before every
 * field (marshal.h:104-108) after the stack budget of its level
 * (marshal.h:129-136). */
typedef struct {
  const plan_t *P;
  const uint8_t *heap;
  uint64_t heap_len;
  uint8_t *out;
  uint64_t cap, pos;
  uint32_t stack_limit, eop;
} ectx;
static int enc_ops(ectx *c, uint32_t pc, obj_t o, uint32_t dbase) {
  const plan_t *P = c->P;
  for (;;) {
    const xdrg_op *op = &P->ops[pc];
    if (op->kind == XDRG_OP_END) return 0;
    if (op->kind == XDRG_OP_JUMP) { pc = op->arg0; continue; }
    if (dbase + op->depth > c->stack_limit) { c->eop = pc; return XDRG_ERR_STACK_PUT; }
    uint64_t need = 4;
    if (op->kind == XDRG_OP_U64) need = 8;
    else if (op->kind == XDRG_OP_OPAQUE) need = op->arg0;
    else if (op->kind == XDRG_OP_VAROPAQUE || op->kind == XDRG_OP_STRING) need = 4 + (uint64_t)o32(o, op->noff + 8);
    if (need > c->cap - c->pos) { c->eop = pc; return XDRG_ERR_OVERFLOW_PUT; }
    uint8_t *w = c->out + c->pos;
    switch (op->kind) {
    case XDRG_OP_U32: case XDRG_OP_ENUM: wr32(w, bswap32(o32(o, op->noff))); c->pos += 4; ++pc; break;
    case XDRG_OP_BOOL: wr32(w, bswap32(o8(o, op->noff) != 0)); c->pos += 4; ++pc; break;
    case XDRG_OP_U64: {
      uint64_t v = o64(o, op->noff);
      wr32(w, bswap32((uint32_t)(v >> 32)));
      wr32(w + 4, bswap32((uint32_t)v));
      c->pos += 8; ++pc; break;
    }
    case XDRG_OP_OPAQUE: {
      uint32_t len = op->arg0;
      obytes(o, op->noff, w, len);
      for (uint64_t k = len; k & 3; ++k) w[k] = 0;
      c->pos += pad4(len); ++pc; break;
    }
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      const uint64_t hoff = o64(o, op->noff);
      const uint32_t len = o32(o, op->noff + 8);
      obj_t h = {c->heap, c->heap_len, hoff};
      wr32(w, bswap32(len));
      obytes(h, 0, w + 4, len);
      for (uint64_t k = len; k & 3; ++k) w[4 + k] = 0;
      c->pos += 4 + pad4(len); ++pc; break;
    }
    case XDRG_OP_UNION: {
      uint32_t d = o32(o, op->noff);
      wr32(w, bswap32(d)); c->pos += 4;
      pc = (uint32_t)union_target(P, op, d);  /* checked by the size pass */
      break;
    }
    case XDRG_OP_VECTOR: {
      /* container save (types.h:374-379): size32 count, then each element */
      const uint64_t eoff = o64(o, op->noff);
      const uint32_t cnt = o32(o, op->noff + 8);
      wr32(w, bswap32(cnt)); c->pos += 4;
      if (!(op->flags & XDRG_F_SUB)) {  /* fixed elements, field by field */
        for (uint32_t i = 0; i < cnt; ++i) {
          obj_t el = {c->heap, c->heap_len, eoff + (uint64_t)i * op->arg1};
          for (uint32_t k = 1; k <= op->arg2; ++k) {
            const xdrg_op *e = &P->ops[pc + k];
            if (dbase + e->depth > c->stack_limit) { c->eop = pc + k; return XDRG_ERR_STACK_PUT; }
            uint32_t wb = elem_wire(e);
            if (wb > c->cap - c->pos) { c->eop = pc + k; return XDRG_ERR_OVERFLOW_PUT; }
            uint8_t *q = c->out + c->pos;
            switch (e->kind) {
            case XDRG_OP_BOOL: wr32(q, bswap32(o8(el, e->noff) != 0)); break;
            case XDRG_OP_U64: {
              uint64_t v = o64(el, e->noff);
              wr32(q, bswap32((uint32_t)(v >> 32)));
              wr32(q + 4, bswap32((uint32_t)v));
              break;
            }
            case XDRG_OP_OPAQUE:
              obytes(el, e->noff, q, e->arg0);
              for (uint64_t b = e->arg0; b & 3; ++b) q[b] = 0;
              break;
            default: wr32(q, bswap32(o32(el, e->noff))); break;
            }
            c->pos += wb;
          }
        }
        pc += 1 + op->arg2;
        break;
      }
      for (uint32_t i = 0; i < cnt; ++i) {
        obj_t el = {c->heap, c->heap_len, eoff + (uint64_t)i * op->arg1};
        int rc = enc_ops(c, op->arg4, el, dbase + op->depth);
        if (rc) return rc;
      }
      ++pc;
      break;
    }
    default: ++pc; break;
    }
  }
}

/* One xdr_generic_put over [out, out+cap) for n records.  Returns 0 or the
 * error code; *erec and *eop receive the failing record and op. */
int xdro_encode(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                const uint8_t *native, uint64_t n, const uint8_t *heap, uint64_t heap_len,
                uint8_t *out, uint64_t cap, uint64_t *offsets, uint32_t stack_limit,
                uint64_t *erec, uint32_t *eop, uint64_t *total) {
  plan_t P = {ops, nops, table, stride, NULL};
  ectx c = {&P, heap, heap_len, out, cap, 0, stack_limit, 0};
  for (uint64_t r = 0; r < n; ++r) {
    const uint8_t *nat = native + r * stride;
    uint32_t err = 0, op_i = 0;
    if (offsets) offsets[r] = c.pos;
    /* xdr_to_opaque sizes the argument pack first (marshal.h:264-268):
     * a bad discriminant throws before any byte is written. */
    rec_size(&P, nat, heap, heap_len, &err, &op_i);
    if (err) { *erec = r; *eop = op_i; return (int)err; }
    obj_t o = {nat, stride, 0};
    int rc = enc_ops(&c, 0, o, 0);
    if (rc) { *erec = r; *eop = c.eop; return rc; }
  }
  if (offsets) offsets[n] = c.pos;
  *total = c.pos;
  return 0;
}

/* Per-record xdr_size (no writes). */
int xdro_sizes(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
               const uint8_t *native, uint64_t n, const uint8_t *heap, uint64_t heap_len,
               uint32_t *sizes, uint64_t *erec, uint32_t *eop) {
  plan_t P = {ops, nops, table, stride, NULL};
  for (uint64_t r = 0; r < n; ++r) {
    uint32_t err = 0, op_i = 0;
    uint64_t s = rec_size(&P, native + r * stride, heap, heap_len, &err, &op_i);
    if (err) { *erec = r; *eop = op_i; return (int)err; }
    sizes[r] = (uint32_t)s;
  }
  return 0;
}

/* depth_checker (xdrpp/depth_checker.h:10-79): per record, the deepest
 * class/container level its walk enters (the record is level 1).
 * check_xdr_depth(r, L) == depths[r] <= L. */
int xdro_depths(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                const uint8_t *native, uint64_t n, const uint8_t *heap, uint64_t heap_len,
                uint32_t *depths, uint64_t *erec, uint32_t *eop) {
  plan_t P = {ops, nops, table, stride, NULL};
  for (uint64_t r = 0; r < n; ++r) {
    szctx c = {&P, heap, heap_len, 0, 0, 0};
    obj_t o = {native + r * stride, stride, 0};
    size_ops(&c, 0, o, 0);
    if (c.err) { *erec = r; *eop = c.eop; return (int)c.err; }
    depths[r] = c.dmax;
  }
  return 0;
}

/* ---------------------------------------------------------------- decode */
/* xdr_generic_get of the object from pc to its END into `nat` (zeroed by
 * the caller); returns 0 or an error code (op in c->eop).  A payload's
 * xdrg_bytes_ref holds its byte offset in the stream (`base`): the decoded
 * heap is the stream itself (heap_out holds a copy).  Element arrays are
 * carved from [ecur, eend) at 8-byte alignment. */
typedef struct {
  const plan_t *P;
  const uint8_t *base, *p, *e;
  uint8_t *heap_out;
  uint64_t ecur, eend;
  uint32_t stack_limit, eop;
} dctx;
static int dec_ops(dctx *c, uint32_t pc, uint8_t *nat, uint32_t dbase) {
  const plan_t *P = c->P;
#define CHECK(nb) do { if ((uint64_t)(nb) > (uint64_t)(c->e - c->p)) { c->eop = pc; return XDRG_ERR_OVERFLOW_GET; } } while (0)
  for (;;) {
    const xdrg_op *op = &P->ops[pc];
    if (op->kind == XDRG_OP_END) return 0;
    if (op->kind == XDRG_OP_JUMP) { pc = op->arg0; continue; }
    if (dbase + op->depth > c->stack_limit) { c->eop = pc; return XDRG_ERR_STACK_GET; }
    switch (op->kind) {
    case XDRG_OP_U32:
      CHECK(4); wr32(nat + op->noff, bswap32(rd32(c->p))); c->p += 4; ++pc; break;
    case XDRG_OP_ENUM: {
      CHECK(4);
      uint32_t v = bswap32(rd32(c->p));
      wr32(nat + op->noff, v); c->p += 4;
      if (!enum_ok(P, op, v)) { c->eop = pc; return XDRG_ERR_INVALID_ENUM; }
      ++pc; break;
    }
    case XDRG_OP_BOOL:
      CHECK(4); nat[op->noff] = rd32(c->p) != 0; c->p += 4; ++pc; break;
    case XDRG_OP_U64: {
      CHECK(8);
      uint64_t hi = bswap32(rd32(c->p)), lo = bswap32(rd32(c->p + 4));
      wr64(nat + op->noff, hi << 32 | lo); c->p += 8; ++pc; break;
    }
    case XDRG_OP_OPAQUE: {
      uint32_t len = op->arg0;
      CHECK(len);
      if (len) {
        memcpy(nat + op->noff, c->p, len);
        c->p += len;
        for (uint64_t k = len; k & 3; ++k)
          if (*c->p++ != 0) { c->eop = pc; return XDRG_ERR_NONZERO_PAD; }
      }
      ++pc; break;
    }
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      CHECK(4);
      uint32_t len = bswap32(rd32(c->p)); c->p += 4;
      CHECK(len);
      if (len > op->arg0) {
        c->eop = pc;
        return op->kind == XDRG_OP_STRING ? XDRG_ERR_XSTRING_BOUND : XDRG_ERR_XVECTOR_BOUND;
      }
      xdrg_bytes_ref ref = {(uint64_t)(c->p - c->base), len, 0};
      if (len) {
        c->p += len;
        for (uint64_t k = len; k & 3; ++k)
          if (*c->p++ != 0) { c->eop = pc; return XDRG_ERR_NONZERO_PAD; }
      }
      memcpy(nat + op->noff, &ref, sizeof ref);
      ++pc; break;
    }
    case XDRG_OP_VECTOR: {
      /* container load (types.h:380-392): count, check_size, elements */
      CHECK(4);
      uint32_t cnt = bswap32(rd32(c->p)); c->p += 4;
      if (cnt > op->arg0) {
        c->eop = pc;
        return (op->flags & XDRG_F_POINTER) ? XDRG_ERR_POINTER_BOUND : XDRG_ERR_XVECTOR_BOUND;
      }
      /* Element area (the kernels' elem_area_ok and sub_kernels.h): valid
       * data always fits; a count the bytes left cannot hold fails here
       * with xdr_overflow -- an element subroutine's before any element,
       * inline elements once the ones the bytes can reach would not fit. */
      {
        const uint64_t rem = (uint64_t)(c->e - c->p);
        const int sub = (op->flags & XDRG_F_SUB) != 0;
        const uint64_t w = sub ? P->minw[op->arg4] : vec_wire(P, pc);
        uint64_t reach = cnt;
        if (!sub && rem / w + 1 < reach) reach = rem / w + 1;
        reach *= op->arg1;
        c->ecur = (c->ecur + 7) & ~7ull;
        if ((sub && (uint64_t)cnt * w > rem) || c->ecur > c->eend || reach > c->eend - c->ecur) {
          c->eop = pc;
          return XDRG_ERR_OVERFLOW_GET;
        }
      }
      xdrg_bytes_ref ref = {c->ecur, cnt, 0};
      memcpy(nat + op->noff, &ref, sizeof ref);
      if (!(op->flags & XDRG_F_SUB)) {  /* fixed elements, field by field */
        for (uint32_t i = 0; i < cnt; ++i) {
          uint8_t *el = c->heap_out + c->ecur + (uint64_t)i * op->arg1;
          memset(el, 0, op->arg1);
          for (uint32_t k = 1; k <= op->arg2; ++k) {
            const xdrg_op *f = &P->ops[pc + k];
            if (dbase + f->depth > c->stack_limit) { c->eop = pc + k; return XDRG_ERR_STACK_GET; }
            uint32_t need = f->kind == XDRG_OP_U64 ? 8u : f->kind == XDRG_OP_OPAQUE ? f->arg0 : 4u;
            if ((uint64_t)need > (uint64_t)(c->e - c->p)) { c->eop = pc + k; return XDRG_ERR_OVERFLOW_GET; }
            switch (f->kind) {
            case XDRG_OP_BOOL: el[f->noff] = rd32(c->p) != 0; break;
            case XDRG_OP_U64: {
              uint64_t hi = bswap32(rd32(c->p)), lo = bswap32(rd32(c->p + 4));
              wr64(el + f->noff, hi << 32 | lo);
              break;
            }
            case XDRG_OP_OPAQUE:
              memcpy(el + f->noff, c->p, f->arg0);
              for (uint64_t q = f->arg0; q & 3; ++q)
                if (c->p[q] != 0) { c->eop = pc + k; return XDRG_ERR_NONZERO_PAD; }
              break;
            default: {
              uint32_t v = bswap32(rd32(c->p));
              wr32(el + f->noff, v);
              if (f->kind == XDRG_OP_ENUM && !enum_ok(P, f, v)) { c->eop = pc + k; return XDRG_ERR_INVALID_ENUM; }
              break;
            }
            }
            c->p += elem_wire(f);
          }
        }
        c->ecur += (uint64_t)cnt * op->arg1;
        pc += 1 + op->arg2;
        break;
      }
      if (cnt) {
        const uint64_t bytes = (uint64_t)cnt * op->arg1, arr = c->ecur;
        memset(c->heap_out + arr, 0, bytes);
        c->ecur += bytes;
        for (uint32_t i = 0; i < cnt; ++i) {
          int rc = dec_ops(c, op->arg4, c->heap_out + arr + (uint64_t)i * op->arg1, dbase + op->depth);
          if (rc) {  /* 1 + the element that failed (the unstager follows it) */
            ref.rsv = i + 1;
            memcpy(nat + op->noff, &ref, sizeof ref);
            return rc;
          }
        }
      }
      ++pc;
      break;
    }
    case XDRG_OP_UNION: {
      CHECK(4);
      uint32_t d = bswap32(rd32(c->p)); c->p += 4;
      if (!enum_ok(P, op, d)) { c->eop = pc; return XDRG_ERR_INVALID_ENUM; }
      int64_t t = union_target(P, op, d);
      if (t < 0) { c->eop = pc; return XDRG_ERR_BAD_DISCRIMINANT; }
      wr32(nat + op->noff, d);
      pc = (uint32_t)t;
      break;
    }
    default: ++pc; break;
    }
  }
#undef CHECK
}

/* Decode one record from [*pp, e) into nat (zero-filled first); element
 * arrays from [ecur, eend).  *pp is advanced. */
static int dec_record(const plan_t *P, const uint8_t **pp, const uint8_t *e, uint8_t *nat,
                      const uint8_t *base, uint8_t *heap_out, uint64_t ecur, uint64_t eend,
                      uint32_t stack_limit, uint32_t *eop) {
  dctx c = {P, base, *pp, e, heap_out, ecur, eend, stack_limit, 0};
  memset(nat, 0, P->stride);
  int rc = dec_ops(&c, 0, nat, 0);
  *pp = c.p;
  *eop = c.eop;
  return rc;
}

/*
 * Fixed or indexed batch decode (see xdrg_decode in include/xdrgpu.h for the
 * contract).  offsets == NULL: one xdr_generic_get over [xdr, xdr+len) for n
 * records, then done().  offsets != NULL: record r is xdr_from_opaque of the
 * slice [off[r], off[r+1]).  heap_out (if given) receives the stream
 * verbatim; every decoded xdrg_bytes_ref points at its payload in it.
 */
static int decode_batch(const plan_t *PP, const uint8_t *xdr, uint64_t len, const uint64_t *offsets,
                        uint64_t n, uint8_t *native, uint8_t *heap_out, uint32_t stack_limit,
                        uint64_t *erec, uint32_t *eop);
int xdro_decode(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                const uint8_t *xdr, uint64_t len, const uint64_t *offsets, uint64_t n,
                uint8_t *native, uint8_t *heap_out, uint32_t stack_limit, uint64_t *erec,
                uint32_t *eop) {
  uint64_t *mw = min_wires(ops, nops, table);
  plan_t P = {ops, nops, table, stride, mw};
  int rc = decode_batch(&P, xdr, len, offsets, n, native, heap_out, stack_limit, erec, eop);
  free(mw);
  return rc;
}
static int decode_batch(const plan_t *PP, const uint8_t *xdr, uint64_t len, const uint64_t *offsets,
                        uint64_t n, uint8_t *native, uint8_t *heap_out, uint32_t stack_limit,
                        uint64_t *erec, uint32_t *eop) {
  const plan_t P = *PP;
  const uint32_t stride = P.stride;
  if (heap_out && len) memcpy(heap_out, xdr, len);
  const uint32_t F = heap_factor(&P);
  const uint64_t ebase = F ? ((len + 15) & ~15ull) : 0;
  if (!offsets) {
    if (len & 3) { *erec = 0; *eop = 0xffffffffu; return XDRG_ERR_SIZE_NOT_MULT4; }
    const uint8_t *p = xdr, *e = xdr + len;
    const int packed = packed_plan(&P);
    uint64_t cur = 0;
    for (uint64_t r = 0; r < n; ++r) {
      const uint64_t a = (uint64_t)(p - xdr);
      uint64_t ec = ebase + (uint64_t)F * a, ee = ebase + (uint64_t)F * len;
      if (packed) {  /* (the record's end is found by its walk: the stream's end bounds it) */
        if (r % 64 == 0) cur = (ebase + (uint64_t)F * a + 7) & ~7ull;
        const uint64_t E = rec_ebytes(&P, xdr, a, len), B = ebudget(F, a, len);
        ec = cur;
        ee = cur + (E < B ? E : B);
        cur = ee;
      }
      int rc = dec_record(&P, &p, e, native + r * stride, xdr, heap_out, ec, ee, stack_limit, eop);
      if (rc) { *erec = r; return rc; }
    }
    if (p != e) { *erec = n; *eop = 0xffffffffu; return XDRG_ERR_TRAILING; }
    return 0;
  }
  const int packed = packed_plan(&P);
  uint64_t cur = 0;  /* packed: the group's bump */
  for (uint64_t r = 0; r < n; ++r) {
    uint64_t a = offsets[r], b = offsets[r + 1];
    if (b < a || b > len) { *erec = r; *eop = 0; return XDRG_ERR_OVERFLOW_GET; }
    if ((b - a) & 3) { *erec = r; *eop = 0xffffffffu; return XDRG_ERR_SIZE_NOT_MULT4; }
    const uint8_t *p = xdr + a, *e = xdr + b;
    uint64_t ec = ebase + (uint64_t)F * a, ee = ebase + (uint64_t)F * b;
    if (packed) {
      if (r % 64 == 0) cur = (ebase + (uint64_t)F * a + 7) & ~7ull;
      const uint64_t E = rec_ebytes(&P, xdr, a, b), B = ebudget(F, a, b);
      ec = cur;
      ee = cur + (E < B ? E : B);
      cur = ee;
    }
    int rc = dec_record(&P, &p, e, native + r * stride, xdr, heap_out, ec, ee, stack_limit, eop);
    if (rc) { *erec = r; return rc; }
    if (p != e) { *erec = r; *eop = 0xffffffffu; return XDRG_ERR_TRAILING; }
  }
  if (offsets[n] != len) { *erec = n; *eop = 0xffffffffu; return XDRG_ERR_TRAILING; }
  return 0;
}

/* ------------------------------------------------------ record-marked messages
 * message_t framing (RFC 5531 record marking): a 4-byte mark
 * BE(size | 0x80000000) before each message's bytes.
 *   xdr_to_msg(r)          marshal.h:252-260, mark by message_t::alloc
 *                          (marshal.cc:15-31)
 *   xdr_from_msg(m, r)     marshal.h:278-284 (xdr_get over m->data())
 *   read_message framing   srpc.cc:29-55; msg_sock's maxmsglen_
 *                          msgsock.cc:85-111
 */
static inline uint32_t mark_code(uint32_t raw, uint64_t body) {
  if (raw & 3) return XDRG_ERR_MSG_SIZE4;       /* srpc.cc:38-39, pre-swap test */
  uint32_t v = bswap32(raw);
  if (!(v & XDRG_MARK_LAST)) return XDRG_ERR_MSG_FRAGMENT; /* srpc.cc:41-45 */
  if ((v & ~XDRG_MARK_LAST) != body) return XDRG_ERR_MSG_MISMATCH;
  return 0;
}

/* n messages, message r = xdr_to_msg(record r). */
int xdro_encode_msgs(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                     const uint8_t *native, uint64_t n, const uint8_t *heap, uint64_t heap_len,
                     uint8_t *out, uint64_t cap, uint64_t *offsets, uint32_t stack_limit,
                     uint64_t *erec, uint32_t *eop, uint64_t *total) {
  plan_t P = {ops, nops, table, stride, NULL};
  uint64_t pos = 0;
  for (uint64_t r = 0; r < n; ++r) {
    const uint8_t *nat = native + r * stride;
    uint32_t err = 0, op_i = 0;
    if (offsets) offsets[r] = pos;
    uint64_t size = rec_size(&P, nat, heap, heap_len, &err, &op_i);  /* xdr_argpack_size */
    if (err) { *erec = r; *eop = op_i; return (int)err; }
    if (4 > cap - pos) { *erec = r; *eop = 0xffffffffu; return XDRG_ERR_OVERFLOW_PUT; }
    wr32(out + pos, bswap32((uint32_t)size | XDRG_MARK_LAST));
    pos += 4;
    uint64_t er = 0, sub = 0;
    int rc = xdro_encode(ops, nops, table, stride, nat, 1, heap, heap_len, out + pos, cap - pos,
                         NULL, stack_limit, &er, eop, &sub);
    if (rc) { *erec = r; return rc; }
    pos += sub;
  }
  if (offsets) offsets[n] = pos;
  *total = pos;
  return 0;
}

/* n messages indexed by offsets (message r = [off[r], off[r+1]), mark
 * included), each decoded as xdr_from_msg. */
static int decode_msgs_batch(const plan_t *PP, const uint8_t *xdr, uint64_t len,
                             const uint64_t *offsets, uint64_t n, uint8_t *native, uint8_t *heap_out,
                             uint32_t stack_limit, uint64_t *erec, uint32_t *eop);
int xdro_decode_msgs(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                     const uint8_t *xdr, uint64_t len, const uint64_t *offsets, uint64_t n,
                     uint8_t *native, uint8_t *heap_out, uint32_t stack_limit, uint64_t *erec,
                     uint32_t *eop) {
  uint64_t *mw = min_wires(ops, nops, table);
  plan_t P = {ops, nops, table, stride, mw};
  int rc = decode_msgs_batch(&P, xdr, len, offsets, n, native, heap_out, stack_limit, erec, eop);
  free(mw);
  return rc;
}
static int decode_msgs_batch(const plan_t *PP, const uint8_t *xdr, uint64_t len,
                             const uint64_t *offsets, uint64_t n, uint8_t *native, uint8_t *heap_out,
                             uint32_t stack_limit, uint64_t *erec, uint32_t *eop) {
  const plan_t P = *PP;
  const uint32_t stride = P.stride;
  if (heap_out && len) memcpy(heap_out, xdr, len);
  const uint32_t F = heap_factor(&P);
  const uint64_t ebase = F ? ((len + 15) & ~15ull) : 0;
  const int packed = packed_plan(&P);
  uint64_t cur = 0;
  for (uint64_t r = 0; r < n; ++r) {
    uint64_t a = offsets[r], b = offsets[r + 1];
    if (b < a || b > len) { *erec = r; *eop = 0; return XDRG_ERR_OVERFLOW_GET; }
    uint32_t c = b - a < 4 ? (uint32_t)XDRG_ERR_MSG_EOF : mark_code(rd32(xdr + a), b - a - 4);
    if (c) { *erec = r; *eop = 0xffffffffu; return (int)c; }
    if ((b - a) & 3) { *erec = r; *eop = 0xffffffffu; return XDRG_ERR_SIZE_NOT_MULT4; }
    const uint8_t *p = xdr + a + 4, *e = xdr + b;
    uint64_t ec = ebase + (uint64_t)F * a, ee = ebase + (uint64_t)F * b;
    if (packed) {
      if (r % 64 == 0) cur = (ebase + (uint64_t)F * a + 7) & ~7ull;
      const uint64_t E = rec_ebytes(&P, xdr, a + 4, b), B = ebudget(F, a, b);
      ec = cur;
      ee = cur + (E < B ? E : B);
      cur = ee;
    }
    int rc = dec_record(&P, &p, e, native + r * stride, xdr, heap_out, ec, ee, stack_limit, eop);
    if (rc) { *erec = r; return rc; }
    if (p != e) { *erec = r; *eop = 0xffffffffu; return XDRG_ERR_TRAILING; }
  }
  if (offsets[n] != len) { *erec = n; *eop = 0xffffffffu; return XDRG_ERR_TRAILING; }
  return 0;
}

/* read_message applied message after message over [s, s+len): offsets[k]
 * = mark k, offsets[count] = len (or the failing mark on an error, which
 * is returned with *erec = count).  A size that is not a multiple of 4
 * stops the index there: xdr_from_msg rejects that message. */
int xdro_index_msgs(const uint8_t *s, uint64_t len, uint32_t maxlen, uint64_t max_msgs,
                    uint64_t *offsets, uint64_t *count, uint64_t *erec) {
  uint64_t pos = 0, k = 0;
  for (;;) {
    offsets[k] = pos;
    *count = k;
    *erec = k;
    if (pos == len) return 0;
    if (k == max_msgs) return XDRG_ERR_MSG_COUNT;
    if (len - pos < 4) return XDRG_ERR_MSG_EOF;            /* srpc.cc:33-37 */
    uint32_t raw = rd32(s + pos);
    if (raw & 3) return XDRG_ERR_MSG_SIZE4;                 /* srpc.cc:38-39 */
    uint32_t v = bswap32(raw);
    if (!(v & XDRG_MARK_LAST)) return XDRG_ERR_MSG_FRAGMENT;  /* srpc.cc:41-45 */
    uint32_t size = v & ~XDRG_MARK_LAST;
    if (size > maxlen) return XDRG_ERR_MSG_TOO_LONG;        /* msgsock.cc:99-111 */
    if (len - pos - 4 < size) return XDRG_ERR_MSG_EOF;      /* srpc.cc:48-52 */
    if (size & 3) return XDRG_ERR_SIZE_NOT_MULT4;           /* marshal.h:152-162 */
    pos += 4 + (uint64_t)size;
    ++k;
  }
}

/* ------------------------------------------------ concatenated records
 * xdrg_index_records restated: the record boundaries xdr_from_opaque
 * (marshal.h:299-306) walks, record after record from byte 0.  A record
 * is parsed for its structure -- lengths, counts, discriminants -- with
 * the checks that make its decode fail (bounds, unknown discriminants,
 * unlisted values of validated enums): where it fails to parse, record k
 * gets [off[k], len) and the rest [len, len).  A record running past
 * a + maxlen (but not past the stream) is XDRG_ERR_INDEX_LONG at k. */
#define RX_BAD 0xffffffffu
#define RX_LONG 0xfffffffeu
typedef struct {
  const plan_t *P;
  const uint8_t *s;
  uint64_t lim;
  uint32_t past;
  uint32_t fcap, fcode; /* element frames the parse follows, and what deeper is */
  int tail;             /* tail containers take their element's frame (the whole-record walk) */
} rxctx;
/* The op after pc, through jumps, is its body's END: a container there,
 * opened in the last element of its own container, takes that element's
 * frame (xdrpp_amd/csrc/sub_kernels.h sub_tail) in the device's
 * whole-record walk (k_rx_long): frames then counts the others.  Its
 * window parses count every frame. */
static int rx_tail(const plan_t *P, uint32_t pc) {
  uint32_t q = pc + 1;
  while (P->ops[q].kind == XDRG_OP_JUMP) q = P->ops[q].arg0;
  return P->ops[q].kind == XDRG_OP_END;
}
/* last: the element being walked is the last of its container */
static uint32_t rx_walk(rxctx *c, uint64_t *pp, uint32_t pc, uint32_t frames, int last) {
  const plan_t *P = c->P;
  uint64_t p = *pp;
  for (;;) {
    const xdrg_op *op = &P->ops[pc];
    if (op->kind == XDRG_OP_END) { *pp = p; return 0; }
    if (op->kind == XDRG_OP_JUMP) { pc = op->arg0; continue; }
    if (op->kind == XDRG_OP_U64) {
      if (c->lim - p < 8) return c->past;
      p += 8; ++pc; continue;
    }
    if (op->kind == XDRG_OP_OPAQUE) {
      if (c->lim - p < op->arg0) return c->past;
      p += pad4(op->arg0); ++pc; continue;
    }
    if (c->lim - p < 4) return c->past;
    const uint32_t v = bswap32(rd32(c->s + p));
    p += 4;
    switch (op->kind) {
    case XDRG_OP_ENUM:
      if (!enum_ok(P, op, v)) return RX_BAD;
      ++pc; break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
      if (v > op->arg0) return RX_BAD;
      if (c->lim - p < v) return c->past;
      p += pad4(v); ++pc; break;
    case XDRG_OP_UNION: {
      if (!enum_ok(P, op, v)) return RX_BAD;
      int64_t t = union_target(P, op, v);
      if (t < 0) return RX_BAD;
      pc = (uint32_t)t;
      break;
    }
    case XDRG_OP_VECTOR:
      if (v > op->arg0) return RX_BAD;
      if (!(op->flags & XDRG_F_SUB)) {
        const uint64_t b = (uint64_t)v * vec_wire(P, pc);
        if (c->lim - p < b) return c->past;
        p += b;
        pc += 1 + op->arg2;
        break;
      }
      /* the device index's windows follow XDRG_INDEX_FRAMES frames: deeper
       * records are left to its long-record walk (or, with a window-sized
       * maxlen, to the caller), as records past the window are; that walk
       * follows XDRG_MAX_FRAMES (deeper: the decode's stack overflow) */
      {
        const int coll = c->tail && frames > 0 && last && rx_tail(P, pc);
        if (v && !coll && frames == c->fcap) return c->fcode;
        for (uint32_t i = 0; i < v; ++i) {
          uint32_t rc = rx_walk(c, &p, op->arg4, coll ? frames : frames + 1, i + 1 == v);
          if (rc) return rc;
        }
      }
      ++pc;
      break;
    default: ++pc; break;
    }
  }
}

int xdro_index_records(const xdrg_op *ops, uint32_t nops, const uint32_t *table, const uint8_t *s,
                       uint64_t len, uint64_t n, uint32_t maxlen, uint64_t *offsets, uint64_t *count,
                       uint64_t *erec) {
  plan_t P = {ops, nops, table, 0, NULL};
  uint64_t p = 0, k = 0;
  /* maxlen past one window (xdrg_index_records' rx_windows): the device
   * walks records of any length and nesting, as this walk then does */
  const int whole = maxlen > XDRG_INDEX_MAX_MSG;
  const uint32_t fcap = whole ? XDRG_MAX_FRAMES : XDRG_INDEX_FRAMES, fcode = whole ? RX_BAD : RX_LONG;
  if (whole) maxlen = UINT32_MAX;
  *count = UINT64_MAX;
  for (; k < n && p < len; ++k) {
    offsets[k] = p;
    const int capped = p + maxlen < len;
    rxctx c = {&P, s, capped ? p + maxlen : len, capped ? RX_LONG : RX_BAD, fcap, fcode, whole};
    uint64_t q = p;
    uint32_t rc = rx_walk(&c, &q, 0, 0, 0);
    if (rc) {
      *count = k;
      for (uint64_t i = k + 1; i <= n; ++i) offsets[i] = len;
      if (rc == RX_LONG) { *erec = k; return XDRG_ERR_INDEX_LONG; }
      return 0;
    }
    p = q;
  }
  offsets[k] = p;
  /* the stream ends at record k (p past len: a ragged stream whose last
   * payload's padding overhangs it -- the unpadded bound test of marshal.h:190
   * passes; the reference's messages are whole words, xdr_generic_get) */
  if (p >= len || k < n) {
    *count = k;
    for (uint64_t i = k + 1; i <= n; ++i) offsets[i] = len;
    return 0;
  }
  /* n records and more bytes: the chain ends at record n unless it parses */
  const int capped = p + maxlen < len;
  rxctx c = {&P, s, capped ? p + maxlen : len, capped ? RX_LONG : RX_BAD, fcap, fcode, whole};
  uint64_t q = p;
  if (rx_walk(&c, &q, 0, 0, 0)) *count = n;
  return 0;
}

/* ------------------------------------------------------------ RPC headers
 * rpc_msg header decode (xdrpp/rpc_msg.x through xdr_get: check(4) per
 * word, opaque body<400>: length, check(size), bound, pad check —
 * marshal.h:163-196, marshal.cc:43-57), then
 *   server: rpc_server_base::dispatch (xdrpp/server.cc:84-107) and the
 *           call_dispatch switch of the service (srpc.h:121-128);
 *   client: check_call_hdr (rpc_msg.cc:115-131) + xid test (srpc.h:61-66).
 * A malformed header keeps only action, err, end and, for a bad
 * discriminant, the union in w[0] (0 _body_t, 1 reply_body, 2
 * rejected_reply); other fields are zero. */
typedef struct { const uint8_t *s; uint64_t p, e; } rcur;

static int rword(rcur *c, uint32_t *v) {
  if (c->e - c->p < 4) return 0;
  *v = bswap32(rd32(c->s + c->p));
  c->p += 4;
  return 1;
}

static uint32_t rauth(rcur *c, uint32_t *len) {
  if (!rword(c, len)) return XDRG_ERR_OVERFLOW_GET;
  if (*len > c->e - c->p) return XDRG_ERR_OVERFLOW_GET;
  if (*len > 400) return XDRG_ERR_XVECTOR_BOUND;
  for (uint64_t j = *len; j & 3; ++j)
    if (c->s[c->p + j]) return XDRG_ERR_NONZERO_PAD;
  c->p += pad4(*len);
  return 0;
}

static uint32_t rwalk(rcur *c, xdrg_rpc_hdr *h) {
  uint32_t v, e;
  if (!rword(c, &h->xid) || !rword(c, &v)) return XDRG_ERR_OVERFLOW_GET;
  h->mtype = (uint8_t)v;
  if (v == 0) { /* CALL: call_body */
    for (int k = 0; k < 5; ++k)
      if (!rword(c, &h->w[k])) return XDRG_ERR_OVERFLOW_GET;
    if ((e = rauth(c, &h->cred_len))) return e;
    if (!rword(c, &h->w[XDRG_RPC_W_VERF_FLAVOR])) return XDRG_ERR_OVERFLOW_GET;
    return rauth(c, &h->verf_len);
  }
  if (v != 1) return XDRG_ERR_BAD_DISCRIMINANT;
  if (!rword(c, &h->w[XDRG_RPC_W_REPLY_STAT])) return XDRG_ERR_OVERFLOW_GET;
  if (h->w[XDRG_RPC_W_REPLY_STAT] == 0) { /* MSG_ACCEPTED: accepted_reply */
    if (!rword(c, &h->w[XDRG_RPC_W_VERF_FLAVOR])) return XDRG_ERR_OVERFLOW_GET;
    if ((e = rauth(c, &h->verf_len))) return e;
    if (!rword(c, &h->w[XDRG_RPC_W_STAT])) return XDRG_ERR_OVERFLOW_GET;
    if (h->w[XDRG_RPC_W_STAT] == 2 &&
        (!rword(c, &h->w[XDRG_RPC_W_LOW]) || !rword(c, &h->w[XDRG_RPC_W_HIGH])))
      return XDRG_ERR_OVERFLOW_GET;
    return 0;
  }
  if (h->w[XDRG_RPC_W_REPLY_STAT] != 1) return XDRG_ERR_BAD_DISCRIMINANT | (1u << 8);
  if (!rword(c, &h->w[XDRG_RPC_W_STAT])) return XDRG_ERR_OVERFLOW_GET;
  if (h->w[XDRG_RPC_W_STAT] == 0)
    return rword(c, &h->w[XDRG_RPC_W_LOW]) && rword(c, &h->w[XDRG_RPC_W_HIGH])
               ? 0 : XDRG_ERR_OVERFLOW_GET;
  if (h->w[XDRG_RPC_W_STAT] != 1) return XDRG_ERR_BAD_DISCRIMINANT | (2u << 8);
  return rword(c, &h->w[XDRG_RPC_W_WHY]) ? 0 : XDRG_ERR_OVERFLOW_GET;
}

static uint32_t rroute(const xdrg_rpc_proc *t, uint32_t nt, xdrg_rpc_hdr *h) {
  const uint32_t P = h->w[XDRG_RPC_W_PROG], V = h->w[XDRG_RPC_W_VERS], Q = h->w[XDRG_RPC_W_PROC];
  int64_t first = -1, last = -1, vhit = 0;
  for (uint32_t i = 0; i < nt; ++i) {
    if (t[i].prog != P) continue;
    if (first < 0) first = i;
    last = i;
    if (t[i].vers == V) {
      vhit = 1;
      if (t[i].proc == Q && !(t[i].flags & XDRG_RPC_PROC_IFACE_ONLY)) return XDRG_RPC_DISPATCH;
    }
  }
  if (first < 0) return XDRG_RPC_PROG_UNAVAIL;
  if (!vhit) {
    h->w[XDRG_RPC_W_LOW] = t[first].vers;
    h->w[XDRG_RPC_W_HIGH] = t[last].vers;
    return XDRG_RPC_PROG_MISMATCH;
  }
  return XDRG_RPC_PROC_UNAVAIL;
}

int xdro_rpc_headers(const uint8_t *s, uint64_t len, const uint64_t *offs, uint64_t n,
                     const xdrg_rpc_proc *procs, uint32_t nprocs, const uint32_t *xids,
                     int client, xdrg_rpc_hdr *out) {
  for (uint64_t i = 0; i < n; ++i) {
    xdrg_rpc_hdr h;
    memset(&h, 0, sizeof h);
    const uint64_t m0 = offs[i], m1 = offs[i + 1];
    uint32_t err;
    if (m1 > len || m1 < m0 + 4 || (m0 & 3)) err = XDRG_ERR_MSG_MISMATCH;
    else if ((m1 - m0) & 3) err = XDRG_ERR_SIZE_NOT_MULT4;
    else {
      rcur c = {s, m0 + 4, m1};
      err = rwalk(&c, &h);
      h.body_off = c.p;
    }
    if (err) {
      memset(&h, 0, sizeof h);
      h.w[0] = err >> 8; /* bad discriminant: 0 _body_t, 1 reply_body, 2 rejected_reply */
      err &= 0xff;
    }
    h.err = (uint8_t)err;
    h.end = m1;
    if (!client) {
      if (err) h.action = XDRG_RPC_DROP_MALFORMED;
      else if (h.mtype != 0) h.action = XDRG_RPC_DROP_NONCALL;
      else if (h.w[XDRG_RPC_W_RPCVERS] != 2) h.action = XDRG_RPC_RPC_MISMATCH;
      else h.action = (uint16_t)rroute(procs, nprocs, &h);
    } else {
      if (err) h.action = XDRG_RPCR_MALFORMED;
      else if (h.mtype != 1) h.action = XDRG_RPCR_NOT_REPLY;
      else if (h.w[XDRG_RPC_W_REPLY_STAT] == 0)
        h.action = h.w[XDRG_RPC_W_STAT] == 0 ? XDRG_RPCR_OK : XDRG_RPCR_ACCEPT_STAT;
      else
        h.action = h.w[XDRG_RPC_W_STAT] == 1 ? XDRG_RPCR_AUTH_STAT : XDRG_RPCR_RPCVERS_MISMATCH;
      if (h.action == XDRG_RPCR_OK && xids && xids[i] != h.xid) h.action = XDRG_RPCR_BAD_XID;
    }
    out[i] = h;
  }
  return 0;
}

/* Error replies (server.cc:8-67) as record-marked messages, message order.
 * Returns 0, or XDRG_ERR_OVERFLOW_PUT with *erec = the first reply that
 * does not fit in cap. */
int xdro_rpc_replies(const xdrg_rpc_hdr *h, uint64_t n, uint8_t *out, uint64_t cap,
                     uint64_t *offs, uint64_t *total, uint64_t *erec) {
  uint64_t pos = 0;
  int rc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t w[9], k = 0, a = h[i].action;
    offs[i] = pos;
    w[k++] = 0; /* mark, below */
    w[k++] = h[i].xid;
    w[k++] = 1; /* REPLY */
    if (a == XDRG_RPC_RPC_MISMATCH) {
      w[k++] = 1; w[k++] = 0; w[k++] = 2; w[k++] = 2;
    } else if (a == XDRG_RPC_AUTH_ERROR) {
      w[k++] = 1; w[k++] = 1; w[k++] = h[i].w[XDRG_RPC_W_WHY];
    } else if (a == XDRG_RPC_PROG_UNAVAIL || a == XDRG_RPC_PROG_MISMATCH ||
               a == XDRG_RPC_PROC_UNAVAIL || a == XDRG_RPC_GARBAGE_ARGS ||
               a == XDRG_RPC_SYSTEM_ERR) {
      w[k++] = 0; w[k++] = 0; w[k++] = 0;
      w[k++] = a == XDRG_RPC_PROG_UNAVAIL ? 1 : a == XDRG_RPC_PROG_MISMATCH ? 2
             : a == XDRG_RPC_PROC_UNAVAIL ? 3 : a == XDRG_RPC_GARBAGE_ARGS ? 4 : 5;
      if (a == XDRG_RPC_PROG_MISMATCH) { w[k++] = h[i].w[XDRG_RPC_W_LOW]; w[k++] = h[i].w[XDRG_RPC_W_HIGH]; }
    } else {
      continue;
    }
    w[0] = (4 * (k - 1)) | XDRG_MARK_LAST;
    if (pos + 4 * k > cap) {
      if (!rc) { rc = XDRG_ERR_OVERFLOW_PUT; *erec = i; }
    } else {
      for (uint32_t j = 0; j < k; ++j) wr32(out + pos + 4 * j, bswap32(w[j]));
    }
    pos += 4 * k;
  }
  offs[n] = pos;
  *total = pos;
  return rc;
}
