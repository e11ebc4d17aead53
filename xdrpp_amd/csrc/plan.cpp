// Host-side plan compiler.
//
// A plan is the flat, wire-ordered field walk that xdr_traits<T>::save
// performs (xdrc/gen_hh.cc:233-243 for structs, :649-660 for unions).  For
// fixed-size plans (no opaque<>/string<>/unions: xdr_traits<T>::
// has_fixed_size, xdrpp/types.h:689-700) the walk is turned into two
// per-word byte-permutation programs:
//   encode: wire word j  <- bytes of the native record (swap32 per 32-bit
//           half, high half first for 64-bit values: xdrpp/marshal.h:65-80)
//   decode: native word k <- bytes of the wire record (the inverse), with
//           padding bytes of the native struct set to zero.
// Variable plans are executed by the device interpreter directly.
#include "plan.h"

#include <algorithm>
#include <cstring>

namespace xdrg {
namespace {

constexpr int kNone = -1;
constexpr int kBoolBase = -1000000;  // marks "bool of word w": kBoolBase - w

uint32_t pad4(uint32_t n) { return (n + 3u) & ~3u; }

bool is_fixed_kind(uint8_t k) {
  return k == XDRG_OP_U32 || k == XDRG_OP_U64 || k == XDRG_OP_BOOL || k == XDRG_OP_ENUM ||
         k == XDRG_OP_OPAQUE;
}

uint32_t native_size(const xdrg_op &op) {
  switch (op.kind) {
  case XDRG_OP_U32: case XDRG_OP_ENUM: case XDRG_OP_UNION: return 4;
  case XDRG_OP_U64: return 8;
  case XDRG_OP_BOOL: return 1;
  case XDRG_OP_OPAQUE: return op.arg0;
  case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: return sizeof(xdrg_bytes_ref);
  default: return 0;
  }
}

// Build a byte-permutation program: out word w takes bytes from the input
// record per `src[4w + i]` (input byte index, kNone for zero, or a bool
// marker).  `prefer_pair` asks for window base (w & ~1) when possible.
// Group path (see plan.h grp_term): G = the fewest records whose input and
// output are both whole 16-byte chunks.  Terms keep their 8-byte windows
// inside the record, so a group's loads stay inside its G records.
void build_group(fixed_prog &pg) {
  pg.grp_G = pg.grp_C = pg.grp_KT = 0;
  pg.grp.clear();
  const uint32_t ib = 4 * pg.in_words, ob = 4 * pg.out_words;
  if (pg.in_words < 2 || pg.out_words == 0) return;
  uint32_t kt = 0;
  for (const term_idx &x : pg.idx) kt = std::max<uint32_t>(kt, x.count);
  if (kt == 0 || kt > 4) return;
  kt = kt <= 1 ? 1 : kt <= 2 ? 2 : 4;
  uint32_t G = 1;
  while ((G * ib) % 16 || (G * ob) % 16) ++G;  // G <= 4
  const uint32_t C = G * ob / 16;
  if (C > 1024) return;
  pg.grp.assign(size_t(C) * 4 * kt, grp_term{0, 0x0C0C0C0Cu});
  for (uint32_t c = 0; c < C; ++c)
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t wg = 4 * c + i, r = wg / pg.out_words, j = wg % pg.out_words;
      const term_idx x = pg.idx[j];
      for (uint32_t q = 0; q < x.count; ++q) {
        const term &t = pg.terms[x.start + q];
        grp_term &g = pg.grp[(size_t(c) * 4 + i) * kt + q];
        g.off = r * ib + 4u * t.src;
        g.sel = t.kind == T_BOOL ? (t.sel | kGrpBool) : t.sel;
        if (t.kind == T_BOOL && t.src + 1u >= pg.in_words) {  // window ends at the record's end
          g.off -= 4u;
          g.sel |= kGrpHi;
        }
      }
    }
  pg.grp_G = G;
  pg.grp_C = C;
  pg.grp_KT = kt;
}

void build_prog(const std::vector<int> &src, uint32_t in_words, uint32_t out_words,
                fixed_prog &pg) {
  pg.in_words = in_words;
  pg.out_words = out_words;
  pg.idx.assign(out_words, {0, 0});
  pg.terms.clear();
  pg.reg.assign(out_words, reg_word{0x0C0C0C0Cu, T_PERM, 0, 0, 0, 0});
  bool reg_ok = true;
  for (uint32_t w = 0; w < out_words; ++w) {
    pg.idx[w].start = uint16_t(pg.terms.size());
    int bytes[4];
    for (int i = 0; i < 4; ++i) bytes[i] = src[4 * w + i];
    // bool terms
    for (int i = 0; i < 4; ++i) {
      if (bytes[i] <= kBoolBase) {
        // marker payload: (src word << 3) | (whole-word test << 2) | src byte
        int sw = kBoolBase - bytes[i];
        term t;
        t.kind = T_BOOL;
        t.src = uint16_t(sw >> 3);
        t.sel = uint32_t(sw & 3) | (uint32_t((sw >> 2) & 1) << 16) | (uint32_t(i) << 8);
        pg.terms.push_back(t);
        bytes[i] = kNone;
        pg.has_bool = true;
      }
    }
    // perm terms: greedily cover the remaining source bytes with 8-byte
    // windows; prefer the aligned pair containing word w.
    bool done[4] = {false, false, false, false};
    for (;;) {
      int m = -1;
      for (int i = 0; i < 4; ++i)
        if (!done[i] && bytes[i] >= 0 && (m < 0 || bytes[i] < m)) m = bytes[i];
      if (m < 0) break;
      uint32_t base = uint32_t(m) / 4;
      uint32_t pair = w & ~1u;
      bool fits_pair = true;
      for (int i = 0; i < 4; ++i)
        if (!done[i] && bytes[i] >= 0 &&
            !(uint32_t(bytes[i]) >= 4 * pair && uint32_t(bytes[i]) < 4 * pair + 8))
          fits_pair = false;
      if (fits_pair && pair + 1 < in_words) base = pair;
      if (base + 1 >= in_words && base > 0) --base;  // window stays inside the record
      uint32_t sel = 0;
      for (int i = 0; i < 4; ++i) {
        uint32_t s = 0x0C;
        if (!done[i] && bytes[i] >= 0 && uint32_t(bytes[i]) >= 4 * base &&
            uint32_t(bytes[i]) < 4 * base + 8) {
          s = uint32_t(bytes[i]) - 4 * base;
          done[i] = true;
        }
        sel |= s << (8 * i);
      }
      pg.terms.push_back(term{T_PERM, uint16_t(base), sel});
    }
    pg.idx[w].count = uint16_t(pg.terms.size() - pg.idx[w].start);
    // register-path eligibility: at most one term; PERM within the pair,
    // BOOL reading the same word index.
    const uint32_t c = pg.idx[w].count;
    if (c == 1) {
      const term &t = pg.terms[pg.idx[w].start];
      if (t.kind == T_PERM) {
        if (t.src != (w & ~1u)) reg_ok = false;
        pg.reg[w].sel = t.sel;
        pg.reg[w].kind = T_PERM;
      } else {
        if (t.src != w) reg_ok = false;
        pg.reg[w].sel = t.sel;
        pg.reg[w].kind = T_BOOL;
      }
    } else if (c > 1) {
      reg_ok = false;
    }
  }
  pg.reg_ok = reg_ok;
  build_group(pg);
}


uint64_t sat_add(uint64_t a, uint64_t b) { return a > UINT64_MAX - b ? UINT64_MAX : a + b; }
uint64_t sat_mul(uint64_t a, uint64_t b) { return a && b > UINT64_MAX / a ? UINT64_MAX : a * b; }

// Regions of a plan: the record's ops up to its END, then one region per
// element subroutine (XDRG_F_SUB), each ending with its own END.  A region's
// ops address a native object of the region's stride: the record's, or the
// element stride of the VECTOR ops that enter it.
struct regions {
  std::vector<uint32_t> id, end, stride;  // per op; per region
};
int split_regions(const xdrg_plan &p, regions &R) {
  const uint32_t n = uint32_t(p.ops.size());
  R.id.assign(n, 0);
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; ++i) {
    R.id[i] = r;
    if (p.ops[i].kind == XDRG_OP_END) {
      R.end.push_back(i);
      ++r;
    }
  }
  if (R.end.empty() || R.end.back() != n - 1) return XDRG_EINVAL;
  R.stride.assign(R.end.size(), 0);
  R.stride[0] = p.stride;
  for (uint32_t i = 0; i < n; ++i) {
    const xdrg_op &op = p.ops[i];
    if (op.kind != XDRG_OP_VECTOR || !(op.flags & XDRG_F_SUB)) continue;
    if (op.arg4 >= n || (op.arg4 && p.ops[op.arg4 - 1].kind != XDRG_OP_END))
      return XDRG_EINVAL;  // a body starts a region
    uint32_t &st = R.stride[R.id[op.arg4]];
    if (st && st != op.arg1) return XDRG_EINVAL;  // one native layout per body
    st = op.arg1;
  }
  for (uint32_t st : R.stride)
    if (!st) return XDRG_EINVAL;  // a region nothing enters
  return XDRG_OK;
}

}  // namespace

int compile_plan(xdrg_plan &p) {
  const uint32_t n = uint32_t(p.ops.size());
  if (n == 0 || p.stride == 0) return XDRG_EINVAL;
  for (const xdrg_op &op : p.ops)
    if (op.kind < XDRG_OP_U32 || op.kind > XDRG_OP_VECTOR) return XDRG_EINVAL;
  regions R;
  if (int rc = split_regions(p, R)) return rc;
  bool fixed = true, saw_end = false;
  p.max_depth = 0;
  p.has_vector = false;
  p.has_sub = false;
  p.heap_factor = 0;
  for (uint32_t i = 0; i < n; ++i) {
    xdrg_op &op = p.ops[i];
    const uint32_t rstride = R.stride[R.id[i]], rend = R.end[R.id[i]];
    if (op.kind == XDRG_OP_END) { saw_end = true; continue; }
    if (op.kind == XDRG_OP_VECTOR) {
      if (op.arg1 == 0) return XDRG_EINVAL;
      if ((op.flags & XDRG_F_POINTER) && op.arg0 != 1) return XDRG_EINVAL;
      if ((op.noff & 7) || uint64_t(op.noff) + sizeof(xdrg_bytes_ref) > rstride) return XDRG_EINVAL;
      if (op.flags & XDRG_F_SUB) {
        // any element type: its body is a subroutine (checked as a region);
        // decoded element arrays take at most stride bytes per element,
        // and distinct elements start at distinct wire words, so the
        // element area needs stride/4 bytes per wire byte, plus the
        // 8-byte alignment of each array (one per count word)
        if (op.arg2 != 0) return XDRG_EINVAL;
        p.heap_factor = std::max<uint32_t>(p.heap_factor, (op.arg1 + 3u) / 4u + 2u);
        p.has_vector = p.has_sub = true;
        if (R.id[i] == 0) p.max_depth = std::max<uint32_t>(p.max_depth, op.depth);
        fixed = false;
        continue;
      }
      // xvector<T,arg0> / pointer<T>: element ops inline in [i+1, i+1+arg2)
      const uint32_t b0 = i + 1, b1 = i + 1 + op.arg2;
      if (op.arg2 == 0 || b1 > rend) return XDRG_EINVAL;
      uint32_t we = 0;
      for (uint32_t k = b0; k < b1; ++k) {
        const xdrg_op &e = p.ops[k];
        if (!is_fixed_kind(e.kind)) return XDRG_EUNSUPPORTED;  // fixed-size elements only
        if (uint64_t(e.noff) + native_size(e) > op.arg1) return XDRG_EINVAL;
        if ((e.kind == XDRG_OP_U32 || e.kind == XDRG_OP_ENUM || e.kind == XDRG_OP_U64) && (e.noff & 3))
          return XDRG_EINVAL;
        if (e.kind == XDRG_OP_ENUM && (e.flags & XDRG_F_VALIDATE) &&
            uint64_t(e.arg0) + e.arg1 > p.table.size())
          return XDRG_EINVAL;
        if (e.depth < op.depth) return XDRG_EINVAL;  // elements sit inside the container level
        we += e.kind == XDRG_OP_U64 ? 8u : e.kind == XDRG_OP_OPAQUE ? pad4(e.arg0) : 4u;
        p.max_depth = std::max<uint32_t>(p.max_depth, e.depth);
      }
      if (we == 0) return XDRG_EUNSUPPORTED;
      op.arg3 = we;  // element wire size, used by the kernels
      p.heap_factor = std::max<uint32_t>(p.heap_factor, (op.arg1 + we - 1) / we + 1u);
      p.has_vector = true;
      p.max_depth = std::max<uint32_t>(p.max_depth, op.depth);
      fixed = false;
      i = b1 - 1;
      continue;
    }
    if (op.kind == XDRG_OP_JUMP) {
      if (op.arg0 > rend || op.arg0 <= i) return XDRG_EINVAL;  // forward, within the region
      fixed = false;
      continue;
    }
    if (!is_fixed_kind(op.kind)) fixed = false;
    if (R.id[i] == 0) p.max_depth = std::max<uint32_t>(p.max_depth, op.depth);
    if (uint64_t(op.noff) + native_size(op) > rstride) return XDRG_EINVAL;
    if ((op.kind == XDRG_OP_ENUM || op.kind == XDRG_OP_UNION) && (op.flags & XDRG_F_VALIDATE) &&
        uint64_t(op.arg0) + op.arg1 > p.table.size())
      return XDRG_EINVAL;
    if (op.kind == XDRG_OP_UNION) {
      if (uint64_t(op.arg2) + 2ull * op.arg3 > p.table.size()) return XDRG_EINVAL;
      for (uint32_t c = 0; c < op.arg3; ++c) {
        uint32_t t = p.table[op.arg2 + 2 * c + 1];
        if (t > rend || t <= i) return XDRG_EINVAL;
      }
      if ((op.flags & XDRG_F_DEFAULT) && (op.arg4 > rend || op.arg4 <= i)) return XDRG_EINVAL;
    }
    if ((op.kind == XDRG_OP_U32 || op.kind == XDRG_OP_ENUM || op.kind == XDRG_OP_UNION) &&
        (op.noff & 3))
      return XDRG_EINVAL;  // natural alignment (C ABI of the xdrc structs)
    if (op.kind == XDRG_OP_U64 && (op.noff & 3)) return XDRG_EINVAL;
    if ((op.kind == XDRG_OP_VAROPAQUE || op.kind == XDRG_OP_STRING) && (op.noff & 7))
      return XDRG_EINVAL;
  }
  if (!saw_end || p.ops.back().kind != XDRG_OP_END) return XDRG_EINVAL;

  p.has_checks = false;
  p.checks.clear();
  {
    // Longest count of var-length fields along any control path (jumps are
    // forward-only, so one reverse sweep over the DAG suffices).
    // Same sweep for the scalar (non-payload) wire words of a record.
    // Computed for fixed plans too: record-marked batches of any plan run
    // on the interpreter kernels, which size themselves with these.
    std::vector<uint32_t> slots(n, 0), words(n, 0);
    std::vector<uint64_t> pieces(n, 0), bytes(n, 0), chunks(n, 0), minw(n, 0);
    for (uint32_t i = n; i-- > 0;) {
      const xdrg_op &op = p.ops[i];
      uint32_t best = 0, bw = 0;
      uint64_t bp = 0, bb = 0, bc = 0, bm = 0;
      switch (op.kind) {
      case XDRG_OP_END: break;
      case XDRG_OP_JUMP:
        best = slots[op.arg0]; bw = words[op.arg0]; bp = pieces[op.arg0]; bb = bytes[op.arg0];
        bc = chunks[op.arg0]; bm = minw[op.arg0];
        break;
      case XDRG_OP_VECTOR: {
        const uint32_t nx = i + 1 + op.arg2;
        best = slots[nx]; bp = pieces[nx]; bc = chunks[nx];
        bw = words[nx] + 1u;  // the count word; elements are unbounded scalar words
        bm = minw[nx] + 4u;   // an empty container
        if (op.flags & XDRG_F_SUB)  // a body entered backwards is recursive: no bound
          bb = sat_add(bytes[nx], sat_add(4, sat_mul(op.arg0, op.arg4 > i ? bytes[op.arg4] : UINT64_MAX)));
        else
          bb = sat_add(bytes[nx], 4ull + uint64_t(op.arg0) * op.arg3);
        break;
      }
      case XDRG_OP_UNION:
        for (uint32_t c = 0; c < op.arg3; ++c) {
          const uint32_t t = p.table[op.arg2 + 2 * c + 1];
          best = std::max(best, slots[t]);
          bw = std::max(bw, words[t]);
          bp = std::max(bp, pieces[t]);
          bb = std::max(bb, bytes[t]);
          bc = std::max(bc, chunks[t]);
          bm = c ? std::min(bm, minw[t]) : minw[t];
        }
        if (op.flags & XDRG_F_DEFAULT) {
          best = std::max(best, slots[op.arg4]);
          bw = std::max(bw, words[op.arg4]);
          bp = std::max(bp, pieces[op.arg4]);
          bb = std::max(bb, bytes[op.arg4]);
          bc = std::max(bc, chunks[op.arg4]);
          bm = op.arg3 ? std::min(bm, minw[op.arg4]) : minw[op.arg4];
        }
        bw += 1;
        bb = sat_add(bb, 4);
        bm += 4;
        break;
      default: {
        const bool var = op.kind == XDRG_OP_VAROPAQUE || op.kind == XDRG_OP_STRING;
        best = slots[i + 1] + (var ? 1u : 0u);
        const uint32_t w = op.kind == XDRG_OP_U64 ? 2u : op.kind == XDRG_OP_OPAQUE ? (op.arg0 + 3u) / 4u : 1u;
        bw = words[i + 1] + w;
        bp = pieces[i + 1] + (var ? (uint64_t(op.arg0) + 255u) / 256u : 0u);
        bb = sat_add(bytes[i + 1], 4ull * w + (var ? (uint64_t(op.arg0) + 3u) & ~3ull : 0u));
        bm = minw[i + 1] + (var ? 4u : 4ull * w);
        bc = chunks[i + 1] + (var ? (uint64_t(op.arg0) + 15u) / 16u : 0u);
        if (var) p.max_slot_len = std::max(p.max_slot_len, op.arg0);
      }
      }
      slots[i] = best;
      words[i] = bw;
      pieces[i] = bp;
      bytes[i] = bb;
      chunks[i] = bc;
      minw[i] = bm;
    }
    // an element subroutine must consume wire bytes (its decoded arrays are
    // bounded by the wire words, see the heap factor above)
    for (xdrg_op &op : p.ops)
      if (op.kind == XDRG_OP_VECTOR && (op.flags & XDRG_F_SUB)) {
        if (minw[op.arg4] < 4) return XDRG_EUNSUPPORTED;
        op.arg3 = uint32_t(std::min<uint64_t>(minw[op.arg4], 0xffffffffu));  // least element wire bytes
      }
    // Nesting of element subroutines: frames[r] = the most frames a walk
    // that enters region r can open below it (UINT32_MAX: a region that can
    // enter itself, i.e. a recursive type).  Past XDRG_SUB_FRAMES the frame
    // walks need their deep passes.
    {
      const uint32_t nreg = uint32_t(R.end.size());
      std::vector<uint32_t> frames(nreg, 0);
      std::vector<uint8_t> state(nreg, 0);  // 0 new, 1 on the DFS path, 2 done
      std::vector<std::pair<uint32_t, uint32_t>> stk;  // (region, next op to look at)
      stk.push_back({0, 0});
      state[0] = 1;
      while (!stk.empty()) {
        auto &top = stk.back();
        const uint32_t reg = top.first, first = reg ? R.end[reg - 1] + 1 : 0;
        uint32_t i = std::max(top.second, first);
        bool pushed = false;
        for (; i < R.end[reg]; ++i) {
          const xdrg_op &op = p.ops[i];
          if (op.kind != XDRG_OP_VECTOR || !(op.flags & XDRG_F_SUB)) continue;
          const uint32_t body = R.id[op.arg4];
          if (state[body] == 1) { frames[reg] = UINT32_MAX; continue; }
          if (state[body] == 0) {
            top.second = i;
            state[body] = 1;
            stk.push_back({body, 0});
            pushed = true;
            break;
          }
          const uint32_t f = frames[body] == UINT32_MAX ? UINT32_MAX : frames[body] + 1;
          frames[reg] = std::max(frames[reg], f);
        }
        if (pushed) continue;
        state[reg] = 2;
        stk.pop_back();
      }
      p.deep = frames[0] > XDRG_SUB_FRAMES;
    }
    // plans whose walks never need the deep passes (no recursive type):
    // each group of 64 records packs its decoded arrays back to back, every
    // array rounded up to 8 bytes (include/xdrgpu.h xdrg_decode_heap_size,
    // oracle/xdr_oracle.c packed_plan); 2 bytes per wire byte more than the
    // record's own arrays need cover that rounding
    p.packed = p.has_vector && !p.deep;
    if (p.packed) p.heap_factor += 2;
    p.max_chunks16 = chunks[0];
    p.max_var_slots = slots[0];
    p.max_scalar_words = words[0];
    p.max_pieces = uint32_t(std::min<uint64_t>(pieces[0], 0xffffffffu));
    p.max_record_bytes = bytes[0];
    p.min_record_bytes = minw[0];
  }
  if (!fixed) {
    p.fixed_size = 0;
    p.path = XDRG_PATH_VAR;
    p.linear = true;
    p.lin_base = 0;
    p.lin_n = 0;
    for (const xdrg_op &op : p.ops) {
      switch (op.kind) {
      case XDRG_OP_U32: case XDRG_OP_BOOL: case XDRG_OP_ENUM: p.lin_base += 4; break;
      case XDRG_OP_U64: p.lin_base += 8; break;
      case XDRG_OP_OPAQUE: p.lin_base += (op.arg0 + 3u) & ~3u; break;
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
        if (p.lin_n == 8) p.linear = false;
        else { p.lin_off[p.lin_n++] = op.noff; p.lin_base += 4; }
        break;
      case XDRG_OP_END: break;
      default: p.linear = false; break;  // UNION, JUMP, VECTOR
      }
    }
    for (const xdrg_op &op : p.ops)
      if (op.kind == XDRG_OP_VAROPAQUE || op.kind == XDRG_OP_STRING || op.kind == XDRG_OP_UNION ||
          op.kind == XDRG_OP_VECTOR ||
          op.kind == XDRG_OP_OPAQUE || (op.kind == XDRG_OP_ENUM && (op.flags & XDRG_F_VALIDATE)))
        p.has_checks = true;
    return XDRG_OK;
  }

  // ---- fixed plan: byte maps
  uint32_t W = 0;
  p.op_wire_off.assign(n, 0);
  for (uint32_t i = 0; i + 1 < n; ++i) {
    const xdrg_op &op = p.ops[i];
    p.op_wire_off[i] = W;
    W += op.kind == XDRG_OP_U64 ? 8 : op.kind == XDRG_OP_OPAQUE ? pad4(op.arg0) : 4;
  }
  p.op_wire_off[n - 1] = W;
  p.fixed_size = W;
  if (p.stride % 4) return XDRG_EUNSUPPORTED;  // word-granular native records
  if (W == 0) return XDRG_EUNSUPPORTED;
  const uint32_t S = p.stride;
  if (S / 4 > 0xffffu || W / 4 > 0xffffu) return XDRG_EUNSUPPORTED;  // u16 word indices

  std::vector<int> enc_src(W, kNone), dec_src(S, kNone);
  for (uint32_t i = 0; i + 1 < n; ++i) {
    const xdrg_op &op = p.ops[i];
    const uint32_t wo = p.op_wire_off[i], no = op.noff;
    switch (op.kind) {
    case XDRG_OP_U32: case XDRG_OP_ENUM:
      for (int k = 0; k < 4; ++k) {  // wire byte k = native byte 3-k (swap32)
        enc_src[wo + k] = int(no + 3 - k);
        dec_src[no + 3 - k] = int(wo + k);
      }
      break;
    case XDRG_OP_U64:
      for (int k = 0; k < 8; ++k) {  // full 64-bit byte reversal
        enc_src[wo + k] = int(no + 7 - k);
        dec_src[no + 7 - k] = int(wo + k);
      }
      break;
    case XDRG_OP_BOOL:
      // wire word = 0/1 in its last (least significant) byte
      enc_src[wo + 3] = kBoolBase - int(no);               // src byte index = no
      dec_src[no] = kBoolBase - int(wo);                    // src word*4
      p.has_bool = true;
      break;
    case XDRG_OP_OPAQUE:
      for (uint32_t k = 0; k < op.arg0; ++k) {
        enc_src[wo + k] = int(no + k);
        dec_src[no + k] = int(wo + k);
      }
      break;
    default: break;
    }
  }
  // Bool markers: encode tests one native byte (the C++ bool), decode tests
  // the whole wire word ("any nonzero is true", types.h:341).  build_prog
  // expects the payload (word << 3) | (whole << 2) | byte.
  for (uint32_t b = 0; b < W; ++b)
    if (enc_src[b] <= kBoolBase) {
      int nb = kBoolBase - enc_src[b];
      enc_src[b] = kBoolBase - ((nb / 4) << 3 | (nb & 3));
    }
  for (uint32_t b = 0; b < S; ++b)
    if (dec_src[b] <= kBoolBase) {
      int wb = kBoolBase - dec_src[b];
      dec_src[b] = kBoolBase - ((wb / 4) << 3 | 4);
    }
  build_prog(enc_src, S / 4, W / 4, p.enc);
  build_prog(dec_src, W / 4, S / 4, p.dec);
  if (p.enc.terms.size() > 0xffffu || p.dec.terms.size() > 0xffffu) return XDRG_EUNSUPPORTED;

  // decode checks
  for (uint32_t i = 0; i + 1 < n; ++i) {
    const xdrg_op &op = p.ops[i];
    if (op.kind == XDRG_OP_OPAQUE && (op.arg0 & 3)) {
      uint32_t last = (p.op_wire_off[i] + op.arg0) / 4;  // word holding the pad
      uint32_t keep = op.arg0 & 3;
      uint32_t mask = ~((1u << (8 * keep)) - 1u);
      p.checks.push_back(check{C_PAD, uint16_t(last), i, mask, 0});
    }
    if (op.kind == XDRG_OP_ENUM && (op.flags & XDRG_F_VALIDATE))
      p.checks.push_back(check{C_ENUM, uint16_t(p.op_wire_off[i] / 4), i, op.arg0, op.arg1});
  }
  p.has_checks = !p.checks.empty();

  const bool identity = (S == W) && (W % 16 == 0) && p.enc.reg_ok && p.dec.reg_ok;
  if (identity) {
    for (const check &c : p.checks) {
      reg_word &rw = p.dec.reg[c.word];  // identity layout: native word == wire word
      if (rw.ck_kind) return XDRG_EUNSUPPORTED;
      rw.ck_kind = c.kind;
      rw.ck_op = c.op;
      rw.ck_a = c.a;
      rw.ck_b = c.b;
    }
  }
  p.path = identity ? XDRG_PATH_FIXED_REG : XDRG_PATH_FIXED_LDS;
  return XDRG_OK;
}

}  // namespace xdrg
