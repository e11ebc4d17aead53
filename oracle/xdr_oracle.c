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

/* xvector<T> / pointer<T> (XDRG_OP_VECTOR): the element's ops follow the
 * op inline, [pc+1, pc+1+arg2); elements are fixed-size. */
static uint32_t elem_wire(const xdrg_op *e) {
  return e->kind == XDRG_OP_U64 ? 8u : e->kind == XDRG_OP_OPAQUE ? pad4(e->arg0) : 4u;
}
static uint32_t vec_wire(const plan_t *P, uint32_t pc) {
  uint32_t w = 0;
  for (uint32_t k = 1; k <= P->ops[pc].arg2; ++k) w += elem_wire(&P->ops[pc + k]);
  return w;
}
/* Decoded element arrays of record r start at align16(len) + F * off[r]
 * (F = 1 + the largest native/wire size ratio of an element type). */
static uint32_t heap_factor(const plan_t *P) {
  uint32_t f = 0;
  for (uint32_t pc = 0; pc < P->nops; ++pc)
    if (P->ops[pc].kind == XDRG_OP_VECTOR) {
      uint32_t we = vec_wire(P, pc), g = (P->ops[pc].arg1 + we - 1) / we + 1;
      if (g > f) f = g;
    }
  return f;
}
uint64_t xdro_decode_heap_size(const xdrg_op *ops, uint32_t nops, uint64_t len) {
  plan_t P = {ops, nops, NULL, 0};
  uint32_t f = heap_factor(&P);
  return f ? ((len + 15) & ~15ull) + (uint64_t)f * len : len;
}

/* xdr_size of one record (xdr_traits<T>::serial_size).  Returns 0 and sets
 * *err and *eop on a bad discriminant. */
static uint64_t rec_size(const plan_t *P, const uint8_t *nat, uint32_t *err, uint32_t *eop) {
  uint64_t s = 0;
  uint32_t pc = 0;
  for (;;) {
    const xdrg_op *op = &P->ops[pc];
    switch (op->kind) {
    case XDRG_OP_U32: case XDRG_OP_BOOL: case XDRG_OP_ENUM: s += 4; ++pc; break;
    case XDRG_OP_U64: s += 8; ++pc; break;
    case XDRG_OP_OPAQUE: s += pad4(op->arg0); ++pc; break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      xdrg_bytes_ref r;
      memcpy(&r, nat + op->noff, sizeof r);
      s += 4 + pad4(r.len);
      ++pc;
      break;
    }
    case XDRG_OP_UNION: {
      int64_t t = union_target(P, op, rd32(nat + op->noff));
      if (t < 0) { *err = XDRG_ERR_BAD_DISCRIMINANT; *eop = pc; return 0; }
      s += 4;
      pc = (uint32_t)t;
      break;
    }
    case XDRG_OP_JUMP: pc = op->arg0; break;
    case XDRG_OP_VECTOR: {
      xdrg_bytes_ref r;
      memcpy(&r, nat + op->noff, sizeof r);
      s += 4 + (uint64_t)r.len * vec_wire(P, pc);
      pc += 1 + op->arg2;
      break;
    }
    default: return s;
    }
  }
}

/* ---------------------------------------------------------------- encode */
/* One xdr_generic_put over [out, out+cap) for n records.  Returns 0 or the
 * error code; *erec and *eop receive the failing record and op. */
int xdro_encode(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                const uint8_t *native, uint64_t n, const uint8_t *heap, uint64_t heap_len,
                uint8_t *out, uint64_t cap, uint64_t *offsets, uint32_t stack_limit,
                uint64_t *erec, uint32_t *eop, uint64_t *total) {
  plan_t P = {ops, nops, table, stride};
  uint64_t pos = 0;
  (void)heap_len;
  for (uint64_t r = 0; r < n; ++r) {
    const uint8_t *nat = native + r * stride;
    uint32_t err = 0, op_i = 0;
    if (offsets) offsets[r] = pos;
    /* xdr_to_opaque sizes the argument pack first (marshal.h:264-268):
     * a bad discriminant throws before any byte is written. */
    rec_size(&P, nat, &err, &op_i);
    if (err) { *erec = r; *eop = op_i; return (int)err; }
    uint32_t pc = 0;
    for (;;) {
      const xdrg_op *op = &ops[pc];
      if (op->kind == XDRG_OP_END) break;
      if (op->kind != XDRG_OP_JUMP && op->depth > stack_limit) {
        *erec = r; *eop = pc; return XDRG_ERR_STACK_PUT;
      }
      uint64_t need = 0;
      switch (op->kind) {
      case XDRG_OP_U32: case XDRG_OP_ENUM: case XDRG_OP_BOOL: case XDRG_OP_UNION:
      case XDRG_OP_VECTOR: need = 4; break;
      case XDRG_OP_U64: need = 8; break;
      case XDRG_OP_OPAQUE: need = op->arg0; break;
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
        xdrg_bytes_ref ref; memcpy(&ref, nat + op->noff, sizeof ref);
        need = 4 + (uint64_t)ref.len;
        break;
      }
      default: break;
      }
      /* check(n): marshal.h:104-108 */
      if (need > cap - pos) { *erec = r; *eop = pc; return XDRG_ERR_OVERFLOW_PUT; }
      switch (op->kind) {
      case XDRG_OP_U32: case XDRG_OP_ENUM:
        wr32(out + pos, bswap32(rd32(nat + op->noff))); pos += 4; ++pc; break;
      case XDRG_OP_BOOL:
        wr32(out + pos, bswap32(nat[op->noff] != 0)); pos += 4; ++pc; break;
      case XDRG_OP_U64: {
        uint64_t v = rd64(nat + op->noff);
        wr32(out + pos, bswap32((uint32_t)(v >> 32)));
        wr32(out + pos + 4, bswap32((uint32_t)v));
        pos += 8; ++pc; break;
      }
      case XDRG_OP_OPAQUE: {
        uint32_t len = op->arg0;
        if (len) {
          memcpy(out + pos, nat + op->noff, len);
          for (uint64_t k = len; k & 3; ++k) out[pos + k] = 0;
          pos += pad4(len);
        }
        ++pc; break;
      }
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
        xdrg_bytes_ref ref; memcpy(&ref, nat + op->noff, sizeof ref);
        wr32(out + pos, bswap32(ref.len)); pos += 4;
        if (ref.len) {
          memcpy(out + pos, heap + ref.off, ref.len);
          for (uint64_t k = ref.len; k & 3; ++k) out[pos + k] = 0;
          pos += pad4(ref.len);
        }
        ++pc; break;
      }
      case XDRG_OP_UNION: {
        uint32_t d = rd32(nat + op->noff);
        wr32(out + pos, bswap32(d)); pos += 4;
        pc = (uint32_t)union_target(&P, op, d);
        break;
      }
      case XDRG_OP_JUMP: pc = op->arg0; break;
      case XDRG_OP_VECTOR: {
        /* container save (types.h:374-379): size32 count, then each element
         * archived field by field (stack + space checks per field) */
        xdrg_bytes_ref ref; memcpy(&ref, nat + op->noff, sizeof ref);
        wr32(out + pos, bswap32(ref.len)); pos += 4;
        for (uint32_t i = 0; i < ref.len; ++i) {
          const uint8_t *el = heap + ref.off + (uint64_t)i * op->arg1;
          for (uint32_t k = 1; k <= op->arg2; ++k) {
            const xdrg_op *e = &ops[pc + k];
            if (e->depth > stack_limit) { *erec = r; *eop = pc + k; return XDRG_ERR_STACK_PUT; }
            uint32_t wb = elem_wire(e);
            if (wb > cap - pos) { *erec = r; *eop = pc + k; return XDRG_ERR_OVERFLOW_PUT; }
            switch (e->kind) {
            case XDRG_OP_BOOL: wr32(out + pos, bswap32(el[e->noff] != 0)); break;
            case XDRG_OP_U64: {
              uint64_t v = rd64(el + e->noff);
              wr32(out + pos, bswap32((uint32_t)(v >> 32)));
              wr32(out + pos + 4, bswap32((uint32_t)v));
              break;
            }
            case XDRG_OP_OPAQUE:
              memcpy(out + pos, el + e->noff, e->arg0);
              for (uint64_t q = e->arg0; q & 3; ++q) out[pos + q] = 0;
              break;
            default: wr32(out + pos, bswap32(rd32(el + e->noff))); break;
            }
            pos += wb;
          }
        }
        pc += 1 + op->arg2;
        break;
      }
      default: ++pc; break;
      }
    }
  }
  if (offsets) offsets[n] = pos;
  *total = pos;
  return 0;
}

/* Per-record xdr_size (no writes). */
int xdro_sizes(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
               const uint8_t *native, uint64_t n, uint32_t *sizes, uint64_t *erec, uint32_t *eop) {
  plan_t P = {ops, nops, table, stride};
  for (uint64_t r = 0; r < n; ++r) {
    uint32_t err = 0, op_i = 0;
    uint64_t s = rec_size(&P, native + r * stride, &err, &op_i);
    if (err) { *erec = r; *eop = op_i; return (int)err; }
    sizes[r] = (uint32_t)s;
  }
  return 0;
}

/* depth_checker (xdrpp/depth_checker.h:10-79): per record, the deepest
 * class/container level its walk enters (the record is level 1; a union
 * and a container count their own level, a non-empty xvector/pointer its
 * element's).  check_xdr_depth(r, L) == depths[r] <= L. */
int xdro_depths(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                const uint8_t *native, uint64_t n, uint32_t *depths, uint64_t *erec,
                uint32_t *eop) {
  plan_t P = {ops, nops, table, stride};
  for (uint64_t r = 0; r < n; ++r) {
    const uint8_t *nat = native + r * stride;
    uint32_t pc = 0, d = 0;
    for (;;) {
      const xdrg_op *op = &P.ops[pc];
      if (op->kind == XDRG_OP_END) break;
      if (op->kind != XDRG_OP_JUMP && op->depth > d) d = op->depth;
      if (op->kind == XDRG_OP_UNION) {
        int64_t t = union_target(&P, op, rd32(nat + op->noff));
        if (t < 0) { *erec = r; *eop = pc; return XDRG_ERR_BAD_DISCRIMINANT; }
        pc = (uint32_t)t;
      } else if (op->kind == XDRG_OP_JUMP) {
        pc = op->arg0;
      } else if (op->kind == XDRG_OP_VECTOR) {
        xdrg_bytes_ref ref;
        memcpy(&ref, nat + op->noff, sizeof ref);
        if (ref.len)
          for (uint32_t k = 1; k <= op->arg2; ++k)
            if (P.ops[pc + k].depth > d) d = P.ops[pc + k].depth;
        pc += 1 + op->arg2;
      } else {
        ++pc;
      }
    }
    depths[r] = d;
  }
  (void)nops;
  return 0;
}

/* ---------------------------------------------------------------- decode */
/* Decode one record from [p, e); returns 0 or an error code (op in *eop).
 * *pp is advanced.  Native record is zero-filled first.  A payload's
 * xdrg_bytes_ref holds its byte offset in the stream (`base`): the decoded
 * heap is the stream itself (xdro_decode copies it to heap_out). */
static int dec_record(const plan_t *P, const uint8_t **pp, const uint8_t *e, uint8_t *nat,
                      const uint8_t *base, uint8_t *heap_out, uint64_t ecur,
                      uint32_t stack_limit, uint32_t *eop) {
  const uint8_t *p = *pp;
  uint32_t pc = 0;
  memset(nat, 0, P->stride);
#define CHECK(nb) do { if ((uint64_t)(nb) > (uint64_t)(e - p)) { *eop = pc; *pp = p; return XDRG_ERR_OVERFLOW_GET; } } while (0)
  for (;;) {
    const xdrg_op *op = &P->ops[pc];
    if (op->kind == XDRG_OP_END) break;
    if (op->kind != XDRG_OP_JUMP && op->depth > stack_limit) {
      *eop = pc; *pp = p; return XDRG_ERR_STACK_GET;
    }
    switch (op->kind) {
    case XDRG_OP_U32:
      CHECK(4); wr32(nat + op->noff, bswap32(rd32(p))); p += 4; ++pc; break;
    case XDRG_OP_ENUM: {
      CHECK(4);
      uint32_t v = bswap32(rd32(p));
      wr32(nat + op->noff, v); p += 4;
      if (!enum_ok(P, op, v)) { *eop = pc; *pp = p; return XDRG_ERR_INVALID_ENUM; }
      ++pc; break;
    }
    case XDRG_OP_BOOL:
      CHECK(4); nat[op->noff] = rd32(p) != 0; p += 4; ++pc; break;
    case XDRG_OP_U64: {
      CHECK(8);
      uint64_t hi = bswap32(rd32(p)), lo = bswap32(rd32(p + 4));
      wr64(nat + op->noff, hi << 32 | lo); p += 8; ++pc; break;
    }
    case XDRG_OP_OPAQUE: {
      uint32_t len = op->arg0;
      CHECK(len);
      if (len) {
        memcpy(nat + op->noff, p, len);
        p += len;
        for (uint64_t k = len; k & 3; ++k)
          if (*p++ != 0) { *eop = pc; *pp = p; return XDRG_ERR_NONZERO_PAD; }
      }
      ++pc; break;
    }
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
      CHECK(4);
      uint32_t len = bswap32(rd32(p)); p += 4;
      CHECK(len);
      if (len > op->arg0) {
        *eop = pc; *pp = p;
        return op->kind == XDRG_OP_STRING ? XDRG_ERR_XSTRING_BOUND : XDRG_ERR_XVECTOR_BOUND;
      }
      xdrg_bytes_ref ref = {(uint64_t)(p - base), len, 0};
      if (len) {
        p += len;
        for (uint64_t k = len; k & 3; ++k)
          if (*p++ != 0) { *eop = pc; *pp = p; return XDRG_ERR_NONZERO_PAD; }
      }
      memcpy(nat + op->noff, &ref, sizeof ref);
      ++pc; break;
    }
    case XDRG_OP_VECTOR: {
      /* container load (types.h:380-392): count, check_size, elements */
      CHECK(4);
      uint32_t cnt = bswap32(rd32(p)); p += 4;
      if (cnt > op->arg0) {
        *eop = pc; *pp = p;
        return (op->flags & XDRG_F_POINTER) ? XDRG_ERR_POINTER_BOUND : XDRG_ERR_XVECTOR_BOUND;
      }
      ecur = (ecur + 7) & ~7ull;
      xdrg_bytes_ref ref = {ecur, cnt, 0};
      memcpy(nat + op->noff, &ref, sizeof ref);
      for (uint32_t i = 0; i < cnt; ++i) {
        uint8_t *el = heap_out + ecur + (uint64_t)i * op->arg1;
        memset(el, 0, op->arg1);
        for (uint32_t k = 1; k <= op->arg2; ++k) {
          const xdrg_op *f = &P->ops[pc + k];
          if (f->depth > stack_limit) { *eop = pc + k; *pp = p; return XDRG_ERR_STACK_GET; }
          uint32_t need = f->kind == XDRG_OP_U64 ? 8u : f->kind == XDRG_OP_OPAQUE ? f->arg0 : 4u;
          if ((uint64_t)need > (uint64_t)(e - p)) { *eop = pc + k; *pp = p; return XDRG_ERR_OVERFLOW_GET; }
          switch (f->kind) {
          case XDRG_OP_BOOL: el[f->noff] = rd32(p) != 0; break;
          case XDRG_OP_U64: {
            uint64_t hi = bswap32(rd32(p)), lo = bswap32(rd32(p + 4));
            wr64(el + f->noff, hi << 32 | lo);
            break;
          }
          case XDRG_OP_OPAQUE:
            memcpy(el + f->noff, p, f->arg0);
            for (uint64_t q = f->arg0; q & 3; ++q)
              if (p[q] != 0) { *eop = pc + k; *pp = p; return XDRG_ERR_NONZERO_PAD; }
            break;
          default: {
            uint32_t v = bswap32(rd32(p));
            wr32(el + f->noff, v);
            if (f->kind == XDRG_OP_ENUM && !enum_ok(P, f, v)) { *eop = pc + k; *pp = p; return XDRG_ERR_INVALID_ENUM; }
            break;
          }
          }
          p += elem_wire(f);
        }
      }
      ecur += (uint64_t)cnt * op->arg1;
      pc += 1 + op->arg2;
      break;
    }
    case XDRG_OP_UNION: {
      CHECK(4);
      uint32_t d = bswap32(rd32(p)); p += 4;
      if (!enum_ok(P, op, d)) { *eop = pc; *pp = p; return XDRG_ERR_INVALID_ENUM; }
      int64_t t = union_target(P, op, d);
      if (t < 0) { *eop = pc; *pp = p; return XDRG_ERR_BAD_DISCRIMINANT; }
      wr32(nat + op->noff, d);
      pc = (uint32_t)t;
      break;
    }
    case XDRG_OP_JUMP: pc = op->arg0; break;
    default: ++pc; break;
    }
  }
#undef CHECK
  *pp = p;
  return 0;
}

/*
 * Fixed or indexed batch decode (see xdrg_decode in include/xdrgpu.h for the
 * contract).  offsets == NULL: one xdr_generic_get over [xdr, xdr+len) for n
 * records, then done().  offsets != NULL: record r is xdr_from_opaque of the
 * slice [off[r], off[r+1]).  heap_out (if given) receives the stream
 * verbatim; every decoded xdrg_bytes_ref points at its payload in it.
 */
int xdro_decode(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                const uint8_t *xdr, uint64_t len, const uint64_t *offsets, uint64_t n,
                uint8_t *native, uint8_t *heap_out, uint32_t stack_limit, uint64_t *erec,
                uint32_t *eop) {
  plan_t P = {ops, nops, table, stride};
  if (heap_out && len) memcpy(heap_out, xdr, len);
  const uint32_t F = heap_factor(&P);
  const uint64_t ebase = F ? ((len + 15) & ~15ull) : 0;
  if (!offsets) {
    if (len & 3) { *erec = 0; *eop = 0xffffffffu; return XDRG_ERR_SIZE_NOT_MULT4; }
    const uint8_t *p = xdr, *e = xdr + len;
    for (uint64_t r = 0; r < n; ++r) {
      int rc = dec_record(&P, &p, e, native + r * stride, xdr, heap_out,
                          ebase + (uint64_t)F * (uint64_t)(p - xdr), stack_limit, eop);
      if (rc) { *erec = r; return rc; }
    }
    if (p != e) { *erec = n; *eop = 0xffffffffu; return XDRG_ERR_TRAILING; }
    return 0;
  }
  for (uint64_t r = 0; r < n; ++r) {
    uint64_t a = offsets[r], b = offsets[r + 1];
    if (b < a || b > len) { *erec = r; *eop = 0; return XDRG_ERR_OVERFLOW_GET; }
    if ((b - a) & 3) { *erec = r; *eop = 0xffffffffu; return XDRG_ERR_SIZE_NOT_MULT4; }
    const uint8_t *p = xdr + a, *e = xdr + b;
    int rc = dec_record(&P, &p, e, native + r * stride, xdr, heap_out, ebase + (uint64_t)F * a,
                        stack_limit, eop);
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
  plan_t P = {ops, nops, table, stride};
  uint64_t pos = 0;
  for (uint64_t r = 0; r < n; ++r) {
    const uint8_t *nat = native + r * stride;
    uint32_t err = 0, op_i = 0;
    if (offsets) offsets[r] = pos;
    uint64_t size = rec_size(&P, nat, &err, &op_i);  /* xdr_argpack_size */
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
int xdro_decode_msgs(const xdrg_op *ops, uint32_t nops, const uint32_t *table, uint32_t stride,
                     const uint8_t *xdr, uint64_t len, const uint64_t *offsets, uint64_t n,
                     uint8_t *native, uint8_t *heap_out, uint32_t stack_limit, uint64_t *erec,
                     uint32_t *eop) {
  plan_t P = {ops, nops, table, stride};
  if (heap_out && len) memcpy(heap_out, xdr, len);
  const uint32_t F = heap_factor(&P);
  const uint64_t ebase = F ? ((len + 15) & ~15ull) : 0;
  for (uint64_t r = 0; r < n; ++r) {
    uint64_t a = offsets[r], b = offsets[r + 1];
    if (b < a || b > len) { *erec = r; *eop = 0; return XDRG_ERR_OVERFLOW_GET; }
    uint32_t c = b - a < 4 ? (uint32_t)XDRG_ERR_MSG_EOF : mark_code(rd32(xdr + a), b - a - 4);
    if (c) { *erec = r; *eop = 0xffffffffu; return (int)c; }
    if ((b - a) & 3) { *erec = r; *eop = 0xffffffffu; return XDRG_ERR_SIZE_NOT_MULT4; }
    const uint8_t *p = xdr + a + 4, *e = xdr + b;
    int rc = dec_record(&P, &p, e, native + r * stride, xdr, heap_out, ebase + (uint64_t)F * a,
                        stack_limit, eop);
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
