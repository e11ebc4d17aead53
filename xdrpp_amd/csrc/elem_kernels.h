// Element helpers shared by the library's interpreted kernels (xdrgpu.hip)
// and by the plan-specialized frame walks (sub_kernels.h, compiled into the
// generated modules too): plan ops read through the scalar cache, union
// case tables, and the inline walk of fixed-size elements of a container.
#pragma once
#include "dev_common.h"

namespace xdrg {
namespace dev {

// ------------------------------------------------------------ var: helpers
// A plan op at a wave-uniform index, read as 8 dwords through the scalar
// cache (s_load_dwordx8) and unpacked.  Reading the struct directly makes
// the compiler fetch the byte fields (kind, flags) with a vector
// global_load_ubyte and wait on it: one memory round trip per op visited.
__device__ __forceinline__ xdrg_op load_op(const xdrg_op *__restrict__ ops, uint32_t i) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(ops) + 8u * i;
  const uint32_t w0 = w[0];
  xdrg_op op;
  op.kind = static_cast<uint8_t>(w0);
  op.flags = static_cast<uint8_t>(w0 >> 8);
  op.depth = static_cast<uint16_t>(w0 >> 16);
  op.noff = w[1];
  op.arg0 = w[2];
  op.arg1 = w[3];
  op.arg2 = w[4];
  op.arg3 = w[5];
  op.arg4 = w[6];
  op.name = w[7];
  return op;
}

// The case table of a union op: (value, target pc) pairs with distinct
// values.  The loop has a wave-uniform trip count and no per-lane exit, so
// the table reads stay scalar (an early per-lane return made them vector
// loads, one memory round trip per union visited).
template <class OP>
__device__ __forceinline__ int union_target(const OP &op, const uint32_t *__restrict__ table, uint32_t d) {
  int t = (op.flags & XDRG_F_DEFAULT) ? static_cast<int>(op.arg4) : -1;
  for (uint32_t i = 0; i < op.arg3; ++i) {
    const uint32_t cv = table[op.arg2 + 2 * i], tg = table[op.arg2 + 2 * i + 1];
    t = cv == d ? static_cast<int>(tg) : t;
  }
  return t;
}

__device__ __forceinline__ void load_ops(xdrg_op *sops, const xdrg_op *__restrict__ ops,
                                         uint32_t nops) {
  const uint32_t *s = reinterpret_cast<const uint32_t *>(ops);
  uint32_t *d = reinterpret_cast<uint32_t *>(sops);
  for (uint32_t i = threadIdx.x; i < nops * 8u; i += blockDim.x) d[i] = s[i];
  __syncthreads();
}

// ------------------------------------------- var: xvector<T> / pointer<T>
// Elements of a VECTOR op (fixed-size element plans; ops [b0, b0+nb)).
// Each element field checks the stack budget (the element's class level)
// and the remaining space before it is archived, as xdr_generic_put/get
// do field by field (marshal.h:110-136, 186-205).
__device__ __forceinline__ uint32_t elem_wire_bytes(const xdrg_op &e) {
  return e.kind == XDRG_OP_U64 ? 8u : e.kind == XDRG_OP_OPAQUE ? (e.arg0 + 3u) & ~3u : 4u;
}

// Encode: native elements from the heap at eoff (stride `es`); put(at, w)
// stores wire word w at stretch offset `at`.
template <typename PUT>
__device__ bool enc_vector_elems(const xdrg_op *__restrict__ ops, uint32_t b0, uint32_t nb,
                                 const uint8_t *__restrict__ heap, uint64_t heap_len, uint64_t eoff,
                                 uint32_t cnt, uint32_t es, uint64_t &pos, uint64_t cap,
                                 uint32_t &at, uint32_t stack_limit, uint64_t r,
                                 unsigned long long *err, const PUT &put) {
  // Elements of at most 16 bytes made of word-aligned scalars and bools are
  // read with one or two loads and taken apart in registers (the per-field
  // path below issues a load per field word).  Wave-uniform test.
  bool staged = (es & 3u) == 0 && es <= 16u;
  for (uint32_t k = 0; k < nb && staged; ++k) {
    const xdrg_op e = load_op(ops, b0 + k);
    staged = e.kind == XDRG_OP_BOOL ||
             ((e.kind == XDRG_OP_U32 || e.kind == XDRG_OP_ENUM || e.kind == XDRG_OP_U64) &&
              (e.noff & 3u) == 0);
  }
  if (staged) {
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint64_t eb = eoff + static_cast<uint64_t>(i) * es;
      uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
      if (eb <= heap_len && es <= heap_len - eb) {  // any byte alignment (ld16u note)
        const uint8_t *q = heap + eb;
        if (es == 4u) {
          w0 = *reinterpret_cast<const uint32_t *>(q);
        } else {
          const uint2 a = *reinterpret_cast<const uint2 *>(q);
          w0 = a.x; w1 = a.y;
          if (es == 12u) w2 = *reinterpret_cast<const uint32_t *>(q + 8);
          else if (es == 16u) { const uint2 c = *reinterpret_cast<const uint2 *>(q + 8); w2 = c.x; w3 = c.y; }
        }
      } else {  // past the heap: bytes read as 0, as unaligned_word does
        w0 = unaligned_word(heap, heap_len, eb);
        if (es > 4u) w1 = unaligned_word(heap, heap_len, eb + 4);
        if (es > 8u) w2 = unaligned_word(heap, heap_len, eb + 8);
        if (es > 12u) w3 = unaligned_word(heap, heap_len, eb + 12);
      }
      auto get = [&](uint32_t j) { return j == 0 ? w0 : j == 1 ? w1 : j == 2 ? w2 : w3; };
      for (uint32_t k = 0; k < nb; ++k) {
        const xdrg_op e = load_op(ops, b0 + k);
        if (e.depth > stack_limit) { report(err, r, b0 + k, XDRG_ERR_STACK_PUT); return false; }
        const uint32_t wb = e.kind == XDRG_OP_U64 ? 8u : 4u;
        if (wb > cap - min(pos, cap)) { report(err, r, b0 + k, XDRG_ERR_OVERFLOW_PUT); return false; }
        const uint32_t j = e.noff >> 2;
        if (e.kind == XDRG_OP_BOOL) {
          put(at, ((get(j) >> (8u * (e.noff & 3u))) & 0xffu) ? 0x01000000u : 0u);
        } else if (e.kind == XDRG_OP_U64) {
          put(at, bswap32(get(j + 1)));
          put(at + 4, bswap32(get(j)));
        } else {
          put(at, bswap32(get(j)));
        }
        at += wb;
        pos += wb;
      }
    }
    return true;
  }
  for (uint32_t i = 0; i < cnt; ++i) {
    const uint64_t eb = eoff + static_cast<uint64_t>(i) * es;
    for (uint32_t k = 0; k < nb; ++k) {
      const xdrg_op e = load_op(ops, b0 + k);
      if (e.depth > stack_limit) { report(err, r, b0 + k, XDRG_ERR_STACK_PUT); return false; }
      const uint32_t wb = elem_wire_bytes(e);
      if (wb > cap - min(pos, cap)) { report(err, r, b0 + k, XDRG_ERR_OVERFLOW_PUT); return false; }
      const uint64_t f = eb + e.noff;
      switch (e.kind) {
      case XDRG_OP_BOOL:
        put(at, (unaligned_word(heap, heap_len, f) & 0xffu) ? 0x01000000u : 0u);
        break;
      case XDRG_OP_U64:
        put(at, bswap32(unaligned_word(heap, heap_len, f + 4)));
        put(at + 4, bswap32(unaligned_word(heap, heap_len, f)));
        break;
      case XDRG_OP_OPAQUE:
        for (uint32_t w = 0; 4u * w < e.arg0; ++w) {
          uint32_t x = unaligned_word(heap, heap_len, f + 4u * w);
          if (4u * w + 4u > e.arg0) x &= keep_mask(e.arg0 - 4u * w);
          put(at + 4u * w, x);
        }
        break;
      default:  // U32, ENUM
        put(at, bswap32(unaligned_word(heap, heap_len, f)));
        break;
      }
      at += wb;
      pos += wb;
    }
  }
  return true;
}

// Decode: wire words through rd(pos); native elements written to `dst`
// (stride `es`, zero-filled first).  p advances; b = end of the record.
template <typename RD>
__device__ bool dec_vector_elems(const xdrg_op *__restrict__ ops, const uint32_t *__restrict__ table,
                                 uint32_t b0, uint32_t nb, uint32_t cnt, uint32_t es, uint8_t *dst,
                                 uint64_t &p, uint64_t b, uint32_t stack_limit, uint64_t r,
                                 unsigned long long *err, RD &rd, uint32_t *done) {
  const bool w4 = (es & 3u) == 0;  // 4-byte stores (dst is 8-aligned)
  // Elements of at most 16 bytes made of word-aligned scalars and bools are
  // assembled in four registers and written with one or two 8-byte stores:
  // the byte-wise path below zero-fills first and stores each field on its
  // own, up to 7 scattered stores per 16-byte element.  The test is on plan
  // ops only, so it is wave-uniform.
  bool staged = w4 && es <= 16u;
  for (uint32_t k = 0; k < nb && staged; ++k) {
    const xdrg_op e = load_op(ops, b0 + k);
    staged = e.kind == XDRG_OP_BOOL ||
             ((e.kind == XDRG_OP_U32 || e.kind == XDRG_OP_ENUM || e.kind == XDRG_OP_U64) &&
              (e.noff & 3u) == 0);
  }
  if (staged) {
    for (uint32_t i = 0; i < cnt; ++i) {
      uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
      auto put = [&](uint32_t j, uint32_t v) {
        w0 |= j == 0 ? v : 0u; w1 |= j == 1 ? v : 0u; w2 |= j == 2 ? v : 0u; w3 |= j == 3 ? v : 0u;
      };
      for (uint32_t k = 0; k < nb; ++k) {
        const xdrg_op e = load_op(ops, b0 + k);
        if (e.depth > stack_limit) { report(err, r, b0 + k, XDRG_ERR_STACK_GET); *done = i; return false; }
        const uint32_t need = e.kind == XDRG_OP_U64 ? 8u : 4u;
        if (b - p < need) { report(err, r, b0 + k, XDRG_ERR_OVERFLOW_GET); *done = i; return false; }
        const uint32_t j = e.noff >> 2;
        if (e.kind == XDRG_OP_BOOL) {
          put(j, (rd(p) != 0u ? 1u : 0u) << (8u * (e.noff & 3u)));
        } else if (e.kind == XDRG_OP_U64) {
          put(j, bswap32(rd(p + 4)));
          put(j + 1, bswap32(rd(p)));
        } else {
          const uint32_t v = bswap32(rd(p));
          put(j, v);
          if (e.kind == XDRG_OP_ENUM && (e.flags & XDRG_F_VALIDATE) && !enum_ok(table, e.arg0, e.arg1, v)) {
            report(err, r, b0 + k, XDRG_ERR_INVALID_ENUM);
            *done = i;
            return false;
          }
        }
        p += need;
      }
      uint8_t *el = dst + static_cast<uint64_t>(i) * es;
      if (es == 4u) {
        st32(el, w0);
      } else {
        *reinterpret_cast<uint2 *>(el) = make_uint2(w0, w1);
        if (es == 12u) st32(el + 8, w2);
        else if (es == 16u) *reinterpret_cast<uint2 *>(el + 8) = make_uint2(w2, w3);
      }
    }
    return true;
  }
  for (uint32_t i = 0; i < cnt; ++i) {
    uint8_t *el = dst + static_cast<uint64_t>(i) * es;
    if (w4) for (uint32_t z = 0; z < es; z += 4) st32(el + z, 0u);
    else for (uint32_t z = 0; z < es; ++z) el[z] = 0;
    for (uint32_t k = 0; k < nb; ++k) {
      const xdrg_op e = load_op(ops, b0 + k);
      if (e.depth > stack_limit) { report(err, r, b0 + k, XDRG_ERR_STACK_GET); *done = i; return false; }
      const uint32_t need = e.kind == XDRG_OP_U64 ? 8u : e.kind == XDRG_OP_OPAQUE ? e.arg0 : 4u;
      if (b - p < need) { report(err, r, b0 + k, XDRG_ERR_OVERFLOW_GET); *done = i; return false; }
      uint8_t *f = el + e.noff;
      switch (e.kind) {
      case XDRG_OP_BOOL:
        f[0] = rd(p) != 0u;
        break;
      case XDRG_OP_U64: {
        const uint32_t hi = bswap32(rd(p)), lo = bswap32(rd(p + 4));
        if (w4) { st32(f, lo); st32(f + 4, hi); }
        else for (int q = 0; q < 4; ++q) { f[q] = uint8_t(lo >> (8 * q)); f[4 + q] = uint8_t(hi >> (8 * q)); }
        break;
      }
      case XDRG_OP_OPAQUE: {
        const uint32_t BL = e.arg0;
        for (uint32_t q = 0; q < BL; q += 4) {
          const uint32_t w = rd(p + q);
          for (uint32_t bb = 0; bb < 4u && q + bb < BL; ++bb) f[q + bb] = uint8_t(w >> (8 * bb));
        }
        if ((BL & 3u) && (rd(p + (BL & ~3u)) & ~keep_mask(BL & 3u))) {
          report(err, r, b0 + k, XDRG_ERR_NONZERO_PAD);
          *done = i;
          return false;
        }
        break;
      }
      default: {  // U32, ENUM
        const uint32_t v = bswap32(rd(p));
        if (w4) st32(f, v);
        else for (int q = 0; q < 4; ++q) f[q] = uint8_t(v >> (8 * q));
        if (e.kind == XDRG_OP_ENUM && (e.flags & XDRG_F_VALIDATE) && !enum_ok(table, e.arg0, e.arg1, v)) {
          report(err, r, b0 + k, XDRG_ERR_INVALID_ENUM);
          *done = i;
          return false;
        }
        break;
      }
      }
      p += elem_wire_bytes(e);
    }
  }
  return true;
}

}  // namespace dev
}  // namespace xdrg
