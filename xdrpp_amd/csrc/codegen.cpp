// Plan-specialized kernel source.
//
// xdrc turns a type into straight-line C++ — xdr_traits<T>::save/load call
// archive() field by field in declaration order (xdrc/gen_hh.cc:212-250,
// unions :575-675).  This back end does the same from a plan: it emits a
// *walker* for var_kernels.h with one block of code per op — the bounds and
// stack checks of xdr_generic_put/get (marshal.h:104-136, :166-205), the
// swaps, the bytes fields — unions as switch statements over their case
// tables, containers as loops.  Compiled (hiprtc at plan time, spec.cpp, or
// ahead of time from the emitted source) the walk carries no op table, no
// per-op dispatch and no wave-uniform sweep: the interpreter's cost.
//
// Control structure comes from the plan's DAG (jumps are forward-only): the
// end of a union is its immediate post-dominator, so every arm is emitted as
// the block from its target to that end.
#include <algorithm>
#include <cstdio>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "plan.h"
#include "spec.h"

namespace xdrg {
namespace {

constexpr uint32_t kNoPc = 0xffffffffu;
constexpr uint32_t kSlotMax = 4;        // chunk-map slots per record (var_kernels.h)
constexpr uint32_t kSlotBytes = 1u << 30;  // longer payloads are copied by their lane
constexpr uint32_t kRegRecordBytes = 128;  // records up to this size are walked from registers
constexpr uint32_t kMaxListWords = 24;     // word-list walks: register budget of emit_words
constexpr uint32_t kSizeUnroll = 4;        // size walk: element loads issued together
constexpr uint32_t kMaxImgWords = 32;      // frame walks: element image in registers

std::string u32(uint32_t v) {
  char b[16];
  snprintf(b, sizeof b, "%uu", v);
  return b;
}

struct gen {
  const xdrg_plan &p;
  std::vector<uint32_t> ipdom;
  std::ostringstream o;
  int ind = 1;
  uint32_t max_slots = 0;  // static chunk-map slots used on the longest path
  uint64_t max_chunks = 0; // 16-byte chunks those slots can hold (per record)
  bool word_list = true;   // every payload takes a slot, no container loop (var_kernels.h WL)
  uint32_t uid = 0;        // names of the element loops of subroutine containers
  uint32_t maxd = 0;       // deepest absolute op depth a walk checks

  explicit gen(const xdrg_plan &plan) : p(plan) { post_dominators(); }

  const xdrg_op &op(uint32_t pc) const { return p.ops[pc]; }
  uint32_t nops() const { return static_cast<uint32_t>(p.ops.size()); }

  // Immediate post-dominators over the control-flow DAG (successors always
  // have a larger pc, so one reverse sweep suffices; END is the exit).
  void post_dominators() {
    const uint32_t n = nops();
    ipdom.assign(n, kNoPc);
    auto meet = [&](uint32_t a, uint32_t b) {
      while (a != b && a != kNoPc && b != kNoPc) {
        if (a < b) a = ipdom[a];
        else b = ipdom[b];
      }
      return a == b ? a : kNoPc;
    };
    for (uint32_t i = n; i-- > 0;) {
      const xdrg_op &o = op(i);
      std::vector<uint32_t> succ;
      switch (o.kind) {
      case XDRG_OP_END: continue;
      case XDRG_OP_JUMP: succ.push_back(o.arg0); break;
      case XDRG_OP_VECTOR: succ.push_back(i + 1 + o.arg2); break;
      case XDRG_OP_UNION:
        for (uint32_t c = 0; c < o.arg3; ++c) succ.push_back(p.table[o.arg2 + 2 * c + 1]);
        if (o.flags & XDRG_F_DEFAULT) succ.push_back(o.arg4);
        break;
      default: succ.push_back(i + 1); break;
      }
      uint32_t d = kNoPc;
      bool first = true;
      for (uint32_t s : succ) {
        d = first ? s : meet(d, s);
        first = false;
      }
      ipdom[i] = d;
    }
  }

  void line(const std::string &s) { o << std::string(2 * ind, ' ') << s << "\n"; }

  // Absolute depth of an op of a body entered with depth offset dadd
  // (include/xdrgpu.h: a subroutine's depths are relative to its VECTOR op)
  std::string depth(const xdrg_op &e, uint32_t dadd) {
    maxd = std::max(maxd, e.depth + dadd);
    return u32(e.depth + dadd);
  }
  // The element at heap offset `eb` of a subroutine container, loaded into
  // registers ew<k> (stride/4 words; heap bytes past `len` read as 0) and
  // seen through the byte pointer e<k>: the body's field reads then have
  // constant offsets, as the record's own.
  std::string load_elem(uint32_t k, const std::string &eb, uint32_t stride, const std::string &heap,
                        const std::string &len) {
    const std::string ew = "ew" + std::to_string(k), e = "e" + std::to_string(k);
    const uint32_t nw = stride / 4;
    line("uint32_t " + ew + "[" + u32(nw) + "];");
    line("if (" + eb + " + " + u32(stride) + " <= " + len + ") {");
    uint32_t q = 0;
    for (; q + 4 <= nw; q += 4)
      line("  { const u32x4 t = ld16u(" + heap + " + " + eb + " + " + u32(4 * q) + "); " + ew + "[" + u32(q) +
           "] = t.x; " + ew + "[" + u32(q + 1) + "] = t.y; " + ew + "[" + u32(q + 2) + "] = t.z; " + ew + "[" +
           u32(q + 3) + "] = t.w; }");
    for (; q < nw; ++q) line("  " + ew + "[" + u32(q) + "] = ld32(" + heap + " + " + eb + " + " + u32(4 * q) + ");");
    line("} else {");
    for (q = 0; q < nw; ++q)
      line("  " + ew + "[" + u32(q) + "] = unaligned_word(" + heap + ", " + len + ", " + eb + " + " + u32(4 * q) + ");");
    line("}");
    line("const uint8_t *" + e + " = reinterpret_cast<const uint8_t *>(" + ew + ");");
    return e;
  }
  // load_elem under a guard, into a named array (the unrolled element
  // loops: several elements' loads issued before any is used)
  std::string load_elem_guarded(const std::string &name, const std::string &guard, const std::string &eb,
                                uint32_t stride, const std::string &heap, const std::string &len) {
    const uint32_t nw = stride / 4;
    line("uint32_t " + name + "w[" + u32(nw) + "];");
    line("if (" + guard + ") {");
    line("  if (" + eb + " + " + u32(stride) + " <= " + len + ") {");
    uint32_t q = 0;
    for (; q + 4 <= nw; q += 4)
      line("    { const u32x4 t = ld16u(" + heap + " + " + eb + " + " + u32(4 * q) + "); " + name + "w[" + u32(q) +
           "] = t.x; " + name + "w[" + u32(q + 1) + "] = t.y; " + name + "w[" + u32(q + 2) + "] = t.z; " + name +
           "w[" + u32(q + 3) + "] = t.w; }");
    for (; q < nw; ++q)
      line("    " + name + "w[" + u32(q) + "] = ld32(" + heap + " + " + eb + " + " + u32(4 * q) + ");");
    line("  } else {");
    for (q = 0; q < nw; ++q)
      line("    " + name + "w[" + u32(q) + "] = unaligned_word(" + heap + ", " + len + ", " + eb + " + " +
           u32(4 * q) + ");");
    line("  }");
    line("}");
    return "reinterpret_cast<const uint8_t *>(" + name + "w)";
  }
  // a body that opens no element subroutine of its own (its walk per
  // element is straight-line code)
  bool body_flat(uint32_t pc) const {
    for (uint32_t q = pc; op(q).kind != XDRG_OP_END; ++q)
      if (op(q).kind == XDRG_OP_VECTOR && (op(q).flags & XDRG_F_SUB)) return false;
    return true;
  }
  // the END that closes the subroutine body starting at pc
  uint32_t body_end(uint32_t pc) const {
    while (op(pc).kind != XDRG_OP_END) ++pc;
    return pc;
  }

  static uint32_t wire_words(const xdrg_op &e) {
    return e.kind == XDRG_OP_U64 ? 2u : e.kind == XDRG_OP_OPAQUE ? (e.arg0 + 3u) / 4u : 1u;
  }
  std::string enum_test(const std::string &v, uint32_t idx, uint32_t cnt) const {
    if (!cnt) return "false";
    std::string t;
    for (uint32_t i = 0; i < cnt; ++i) t += (i ? " || " : "") + v + " == " + u32(p.table[idx + i]);
    return "(" + t + ")";
  }
  // distinct case targets of a union, in table order, with their values
  std::vector<std::pair<uint32_t, std::vector<uint32_t>>> arms(const xdrg_op &u) const {
    std::vector<std::pair<uint32_t, std::vector<uint32_t>>> out;
    for (uint32_t c = 0; c < u.arg3; ++c) {
      const uint32_t v = p.table[u.arg2 + 2 * c], t = p.table[u.arg2 + 2 * c + 1];
      auto it = std::find_if(out.begin(), out.end(), [&](auto &a) { return a.first == t; });
      if (it == out.end()) out.push_back({t, {v}});
      else it->second.push_back(v);
    }
    return out;
  }

  // ------------------------------------------------------------------ size
  // xdr_size (types.h:240-244; unions gen_hh.cc:639-648): returns through s.
  void size_block(uint32_t pc, uint32_t stop, const std::string &base) {
    while (pc != stop) {
      const xdrg_op &e = op(pc);
      const std::string f = base + " + " + u32(e.noff);
      switch (e.kind) {
      case XDRG_OP_END: return;
      case XDRG_OP_JUMP: pc = e.arg0; continue;
      case XDRG_OP_U32: case XDRG_OP_ENUM: case XDRG_OP_BOOL: line("s += 4;"); break;
      case XDRG_OP_U64: line("s += 8;"); break;
      case XDRG_OP_OPAQUE: line("s += " + u32((e.arg0 + 3u) & ~3u) + ";"); break;
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
        line("s += 4ull + ((static_cast<uint64_t>(ld32(" + f + " + 8)) + 3u) & ~3ull);");
        break;
      case XDRG_OP_VECTOR:
        if (e.flags & XDRG_F_SUB) {  // element subroutine: the body's size per element
          const uint32_t k = uid++;
          line("{");
          ++ind;
          line("const uint64_t eoff" + std::to_string(k) + " = *reinterpret_cast<const uint64_t *>(" + f + ");");
          line("const uint32_t cnt" + std::to_string(k) + " = ld32(" + f + " + 8);");
          line("s += 4;");
          const std::string K = std::to_string(k);
          if (body_flat(e.arg4) && e.arg1 <= 64u) {
            // kSizeUnroll elements at a time, their loads first: the
            // element walks do not wait on one load after another
            line("for (uint32_t i" + K + " = 0; i" + K + " < cnt" + K + "; i" + K + " += " + u32(kSizeUnroll) + ") {");
            ++ind;
            std::vector<std::string> els;
            for (uint32_t j = 0; j < kSizeUnroll; ++j) {
              const std::string eb = "(eoff" + K + " + static_cast<uint64_t>(i" + K + " + " + u32(j) + ") * " +
                                     u32(e.arg1) + ")";
              els.push_back(load_elem_guarded("u" + K + "_" + std::to_string(j), "i" + K + " + " + u32(j) + " < cnt" + K,
                                              eb, e.arg1, "heap", "heap_len"));
            }
            for (uint32_t j = 0; j < kSizeUnroll; ++j) {
              line("if (i" + K + " + " + u32(j) + " < cnt" + K + ") {");
              ++ind;
              size_block(e.arg4, body_end(e.arg4), els[j]);
              --ind;
              line("}");
            }
            --ind;
            line("}");
          } else {
            line("for (uint32_t i" + K + " = 0; i" + K + " < cnt" + K + "; ++i" + K + ") {");
            ++ind;
            const std::string eb = "(eoff" + K + " + static_cast<uint64_t>(i" + K + ") * " + u32(e.arg1) + ")";
            const std::string el = load_elem(k, eb, e.arg1, "heap", "heap_len");
            size_block(e.arg4, body_end(e.arg4), el);
            --ind;
            line("}");
          }
          --ind;
          line("}");
          ++pc;
          continue;
        }
        line("s += 4ull + static_cast<uint64_t>(ld32(" + f + " + 8)) * " + u32(e.arg3) + ";");
        pc += 1 + e.arg2;
        continue;
      case XDRG_OP_UNION: {
        const uint32_t end = ipdom[pc];
        line("s += 4;");
        line("switch (ld32(" + f + ")) {");
        for (auto &a : arms(e)) {
          std::string lab;
          for (uint32_t v : a.second) lab += "case " + u32(v) + ": ";
          line(lab + "{");
          ++ind;
          size_block(a.first, end, base);
          --ind;
          line("} break;");
        }
        line("default: {");
        ++ind;
        if (e.flags & XDRG_F_DEFAULT) size_block(e.arg4, end, base);
        else line("bad_op = " + u32(pc) + "; return s;");
        --ind;
        line("} break;");
        line("}");
        pc = end;
        continue;
      }
      default: break;
      }
      ++pc;
    }
  }

  // ----------------------------------------------------- record parse
  // The record-start parse of the plain-stream index (rx_len of
  // xdrgpu.hip, straight-line): lengths, counts and discriminants only,
  // with every check that makes a decode fail.  Returns through p, or
  // `past` when the record runs past lim, or RX_BAD.
  // Runs of fixed-size fields are not tested one by one: their bytes (pend)
  // join the next read's bound test, or one test at the block's end (chk:
  // the most any of the skipped tests asked; nothing between them can fail
  // otherwise, so the record fails the same way).  The parse is a divergent
  // walk per lane: every instruction saved counts once per union arm.
  // With rx_sticky set the same parse runs without early returns (the
  // staged-stretch parse, rlen_st): the first failure is kept in r and the
  // rest of the record runs on (its reads clamped into the stretch, its
  // element loops stopped), so lanes rejoin at every test instead of
  // leaving the wave's execution mask one by one.
  bool rx_sticky = false;
  void fail(const std::string &cond, const std::string &code) {
    if (rx_sticky) line("r = (r == 0u && (" + cond + ")) ? " + code + " : r;");
    else line("if (" + cond + ") return " + code + ";");
  }
  void rx_block(uint32_t pc, uint32_t stop) {
    uint32_t pend = 0, chk = 0;
    auto need = [&](const std::string &n) { fail("lim - p < " + n, "past"); };
    auto skip = [&](uint32_t least, uint32_t adv) {
      chk = std::max(chk, pend + least);
      pend += adv;
    };
    auto flush = [&]() {
      if (chk) need(u32(chk));
      if (pend) line("p += " + u32(pend) + ";");
      pend = chk = 0;
    };
    auto word = [&]() {
      need(u32(std::max(chk, pend + 4)));
      line("{ const uint32_t v = bswap32(rd." + std::string(rx_sticky ? "atc(" : "at(") +
           (pend ? "p + " + u32(pend) : std::string("p")) + ")); p += " + u32(pend + 4) + ";");
      pend = chk = 0;
    };
    while (pc != stop) {
      const xdrg_op &e = op(pc);
      switch (e.kind) {
      case XDRG_OP_END: flush(); return;
      case XDRG_OP_JUMP: pc = e.arg0; continue;
      case XDRG_OP_U64: skip(8, 8); break;
      case XDRG_OP_OPAQUE: skip(e.arg0, (e.arg0 + 3u) & ~3u); break;
      case XDRG_OP_U32: case XDRG_OP_BOOL: skip(4, 4); break;
      case XDRG_OP_ENUM:
        if (e.flags & XDRG_F_VALIDATE) {
          word();
          ind += 2;
          fail("!" + enum_test("v", e.arg0, e.arg1), "RX_BAD");
          ind -= 2;
          line("}");
        } else {
          skip(4, 4);
        }
        break;
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
        word();
        ind += 2;
        fail("v > " + u32(e.arg0), "RX_BAD");
        fail("lim - p < v", "past");
        ind -= 2;
        line("  p += static_cast<U>((static_cast<uint64_t>(v) + 3u) & ~3ull); }");
        break;
      case XDRG_OP_VECTOR:
        if (e.flags & XDRG_F_SUB) {  // each element parsed by its body
          const std::string k = std::to_string(uid++);
          word();
          ind += 2;
          fail("v > " + u32(e.arg0), "RX_BAD");
          fail("(lim - p) / " + u32(e.arg3) + " < v", "past");  // the decode's least-wire check
          ind -= 2;
          line("  for (uint32_t i" + k + " = 0; i" + k + " < v" + (rx_sticky ? " && r == 0u" : "") + "; ++i" + k +
               ") {");
          ind += 2;
          rx_block(e.arg4, body_end(e.arg4));
          ind -= 2;
          line("  }");
          line("}");
          ++pc;
          continue;
        }
        word();
        ind += 2;
        fail("v > " + u32(e.arg0), "RX_BAD");
        line("const uint64_t b = static_cast<uint64_t>(v) * " + u32(e.arg3) + ";");
        fail("static_cast<uint64_t>(lim - p) < b", "past");
        ind -= 2;
        line("  p += static_cast<U>(b); }");
        pc += 1 + e.arg2;
        continue;
      case XDRG_OP_UNION: {
        const uint32_t end = ipdom[pc];
        word();
        ind += 2;
        if (e.flags & XDRG_F_VALIDATE) fail("!" + enum_test("v", e.arg0, e.arg1), "RX_BAD");
        ind -= 2;
        line("  switch (v) {");
        for (auto &a : arms(e)) {
          std::string lab;
          for (uint32_t v : a.second) lab += "case " + u32(v) + ": ";
          line("  " + lab + "{");
          ind += 2;
          rx_block(a.first, end);
          ind -= 2;
          line("  } break;");
        }
        line("  default: {");
        ind += 2;
        if (e.flags & XDRG_F_DEFAULT) rx_block(e.arg4, end);
        else if (rx_sticky) line("r = r ? r : RX_BAD;");
        else line("return RX_BAD;");
        ind -= 2;
        line("  } break;");
        line("  }");
        line("}");
        pc = end;
        continue;
      }
      default: break;
      }
      ++pc;
    }
    flush();
  }
  // Packed element areas: the bytes a record's arrays take, each rounded up
  // to 8 (oracle/xdr_oracle.c rec_ebytes, var_kernels.h packed_area) -- a
  // walk of its lengths, counts and discriminants that stops (returns E)
  // where the structure stops parsing.  Element subroutines (non-recursive:
  // packed plans are never deep) are walked inline per element.  At the
  // record's level (top) the walk stops as soon as no container can follow
  // (jumps go forward only, so none at a later pc means none reachable): E
  // is final there, and containertest's shares skip its element bodies and
  // strings altogether.
  bool region_has_vector(uint32_t start) const {
    for (uint32_t i = start; i < nops() && op(i).kind != XDRG_OP_END; ++i)
      if (op(i).kind == XDRG_OP_VECTOR) return true;
    return false;
  }
  bool vector_from(uint32_t pc) const { return region_has_vector(pc); }  // the record region: [pc, its END)
  void eb_block(uint32_t pc, uint32_t stop, bool top = false) {
    auto need = [&](const std::string &n) { line("if (b - q < " + n + ") return E;"); };
    auto word = [&]() { need("4"); line("{ const uint32_t v = bswap32(rd(q)); q += 4;"); };
    while (pc != stop) {
      if (top && !vector_from(pc)) {
        line("return E;");
        return;
      }
      const xdrg_op &e = op(pc);
      switch (e.kind) {
      case XDRG_OP_END: return;
      case XDRG_OP_JUMP: pc = e.arg0; continue;
      case XDRG_OP_U64: need("8"); line("q += 8;"); break;
      case XDRG_OP_OPAQUE: need(u32(e.arg0)); line("q += " + u32((e.arg0 + 3u) & ~3u) + ";"); break;
      case XDRG_OP_U32: case XDRG_OP_BOOL: case XDRG_OP_ENUM: need("4"); line("q += 4;"); break;
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
        word();
        line("  if (v > " + u32(e.arg0) + " || v > b - q) return E;");
        line("  q += (static_cast<uint64_t>(v) + 3u) & ~3ull; }");
        break;
      case XDRG_OP_VECTOR:
        word();
        line("  if (v > " + u32(e.arg0) + ") return E;");
        line("  const uint64_t left = b - q;");
        if (e.flags & XDRG_F_SUB) {
          // an element subroutine: its array when the bytes left can hold
          // the count (arg3 = the least an element consumes), then each
          // element's own arrays (the body inline)
          line("  if (left < static_cast<uint64_t>(v) * " + u32(e.arg3) + ") return E;");
          line("  E += (static_cast<uint64_t>(v) * " + u32(e.arg1) + " + 7u) & ~7ull;");
          if (top && !region_has_vector(e.arg4) && !vector_from(pc + 1)) {  // nothing after adds to E
            line("  return E; }");
            return;
          }
          line("  for (uint32_t i = 0; i < v; ++i) {");
          ind += 4;
          eb_block(e.arg4, body_end(e.arg4));
          ind -= 4;
          line("  } }");
          ++pc;
          continue;
        }
        line("  E += (min<uint64_t>(v, left / " + u32(e.arg3) + " + 1u) * " + u32(e.arg1) + " + 7u) & ~7ull;");
        line("  if (left < static_cast<uint64_t>(v) * " + u32(e.arg3) + ") return E;");
        line("  q += static_cast<uint64_t>(v) * " + u32(e.arg3) + "; }");
        pc += 1 + e.arg2;
        continue;
      case XDRG_OP_UNION: {
        const uint32_t end = ipdom[pc];
        word();
        line("  switch (v) {");
        for (auto &a : arms(e)) {
          std::string lab;
          for (uint32_t v : a.second) lab += "case " + u32(v) + ": ";
          line("  " + lab + "{");
          ind += 2;
          eb_block(a.first, end, top);
          ind -= 2;
          line("  } break;");
        }
        line("  default: {");
        ind += 2;
        if (e.flags & XDRG_F_DEFAULT) eb_block(e.arg4, end, top);
        else line("return E;");
        ind -= 2;
        line("  } break;");
        line("  }");
        line("}");
        pc = end;
        continue;
      }
      default: break;
      }
      ++pc;
    }
  }
  // The first op whose word is checked (every op before it fixed-size, no
  // branch) and the test of that word: what the index loads for every
  // candidate start before parsing it (run_index in xdrgpu.hip finds the
  // same op).
  // Least bytes the record needs after that word given its value v: a
  // container's count times the least an element takes, a payload's length.
  std::string first_len() {
    for (uint32_t pc = 0; pc < nops(); ++pc) {
      const xdrg_op &o = op(pc);
      if (o.kind == XDRG_OP_END || o.kind == XDRG_OP_JUMP) break;
      if (o.kind == XDRG_OP_U64 || o.kind == XDRG_OP_OPAQUE || o.kind == XDRG_OP_U32 || o.kind == XDRG_OP_BOOL ||
          (o.kind == XDRG_OP_ENUM && !(o.flags & XDRG_F_VALIDATE)))
        continue;
      if (o.kind == XDRG_OP_VECTOR) return "static_cast<uint64_t>(v) * " + u32(o.arg3);
      if (o.kind == XDRG_OP_VAROPAQUE || o.kind == XDRG_OP_STRING) return "static_cast<uint64_t>(v)";
      return "0";
    }
    return "0";
  }
  std::string first_test(uint32_t pc0 = 0, const std::string &x = "v") {
    for (uint32_t pc = pc0; pc < nops(); ++pc) {
      const xdrg_op &o = op(pc);
      if (o.kind == XDRG_OP_END || o.kind == XDRG_OP_JUMP) break;
      if (o.kind == XDRG_OP_U64 || o.kind == XDRG_OP_OPAQUE || o.kind == XDRG_OP_U32 || o.kind == XDRG_OP_BOOL ||
          (o.kind == XDRG_OP_ENUM && !(o.flags & XDRG_F_VALIDATE)))
        continue;
      if (o.kind == XDRG_OP_ENUM) return enum_test(x, o.arg0, o.arg1);
      if (o.kind == XDRG_OP_UNION) {
        if (o.flags & XDRG_F_DEFAULT) return (o.flags & XDRG_F_VALIDATE) ? enum_test(x, o.arg0, o.arg1) : "true";
        std::string t;
        for (auto &a : arms(o))
          for (uint32_t v : a.second) t += (t.empty() ? "" : " || ") + x + " == " + u32(v);
        if (t.empty()) t = "false";
        return (o.flags & XDRG_F_VALIDATE) ? "(" + enum_test(x, o.arg0, o.arg1) + " && (" + t + "))" : "(" + t + ")";
      }
      return x + " <= " + u32(o.arg0);  // VAROPAQUE, STRING, VECTOR
    }
    return "true";
  }
  // The word after the first checked one, w, given that one's value v: when
  // the record starts with a container of element-subroutine elements whose
  // body opens with a checked field, a nonempty count's next word is that
  // field of the first element (containertest: the union's discriminant).
  std::string second_test() {
    for (uint32_t pc = 0; pc < nops(); ++pc) {
      const xdrg_op &o = op(pc);
      if (o.kind == XDRG_OP_END || o.kind == XDRG_OP_JUMP) break;
      if (o.kind == XDRG_OP_U64 || o.kind == XDRG_OP_OPAQUE || o.kind == XDRG_OP_U32 || o.kind == XDRG_OP_BOOL ||
          (o.kind == XDRG_OP_ENUM && !(o.flags & XDRG_F_VALIDATE)))
        continue;
      if (o.kind != XDRG_OP_VECTOR || !(o.flags & XDRG_F_SUB)) return "true";
      const xdrg_op &b = op(o.arg4);  // the body's first op must be the checked one (no offset)
      const bool checked = b.kind == XDRG_OP_UNION || (b.kind == XDRG_OP_ENUM && (b.flags & XDRG_F_VALIDATE)) ||
                           b.kind == XDRG_OP_VAROPAQUE || b.kind == XDRG_OP_STRING || b.kind == XDRG_OP_VECTOR;
      if (!checked) return "true";
      return "(v == 0u || " + first_test(o.arg4, "w") + ")";
    }
    return "true";
  }

  // ---------------------------------------------------------------- encode
  // xdr_generic_put field by field (marshal.h:84-137).  Returns the static
  // slots used after the block (slots count along the path); `words` = the
  // most scalar words a path through the block puts.
  uint32_t enc_block(uint32_t pc, uint32_t stop, uint32_t slot, uint64_t &chunks, uint32_t &words,
                     const std::string &base = "nat", uint32_t dadd = 0) {
    while (pc != stop) {
      const xdrg_op &e = op(pc);
      const std::string f = base + " + " + u32(e.noff), P = u32(pc), D = depth(e, dadd);
      switch (e.kind) {
      case XDRG_OP_END: return slot;
      case XDRG_OP_JUMP: pc = e.arg0; continue;
      case XDRG_OP_U32: case XDRG_OP_ENUM:
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line("c.put(bswap32(ld32(" + f + ")));");
        words += 1;
        break;
      case XDRG_OP_BOOL:
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line("c.put(" + base + "[" + u32(e.noff) + "] ? 0x01000000u : 0u);");
        words += 1;
        break;
      case XDRG_OP_U64:
        line("if (!c.field(" + P + ", " + D + ", 8)) return false;");
        line("c.put(bswap32(ld32(" + f + " + 4)));");
        line("c.put(bswap32(ld32(" + f + ")));");
        words += 2;
        break;
      case XDRG_OP_OPAQUE: {
        line("if (!c.field(" + P + ", " + D + ", " + u32(e.arg0) + ")) return false;");
        words += (e.arg0 + 3u) / 4u;
        for (uint32_t k = 0; 4 * k < e.arg0; ++k) {
          std::string w;
          for (uint32_t b = 0; b < 4 && 4 * k + b < e.arg0; ++b)
            w += std::string(b ? " | " : "") + "(uint32_t(" + base + "[" + u32(e.noff + 4 * k + b) + "]) << " +
                 std::to_string(8 * b) + ")";
          line("c.put(" + w + ");");
        }
        break;
      }
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
        line("{");
        ++ind;
        line("const uint32_t len = ld32(" + f + " + 8);");
        line("if (!c.field(" + P + ", " + D + ", 4ull + len)) return false;");
        line("c.put(bswap32(len));");
        words += 1;
        line("const uint64_t src = *reinterpret_cast<const uint64_t *>(" + f + ");");
        if (slot < kSlotMax) {
          const uint32_t cap = std::min(e.arg0, kSlotBytes);
          if (e.arg0 > kSlotBytes) {
            line("if (len > " + u32(kSlotBytes) + ") c.copy(src, len); else c.template slot<" +
                 std::to_string(slot) + ">(src, len);");
            word_list = false;
          } else {
            line("c.template slot<" + std::to_string(slot) + ">(src, len);");
          }
          chunks += (cap + 15u) / 16u;
          ++slot;
        } else {
          line("c.copy(src, len);");
          word_list = false;
        }
        --ind;
        line("}");
        break;
      }
      case XDRG_OP_UNION: {
        const uint32_t end = ipdom[pc];
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line("{");
        ++ind;
        line("const uint32_t d = ld32(" + f + ");");
        line("c.put(bswap32(d));");
        words += 1;
        line("switch (d) {");
        uint32_t smax = slot, wmax = words;
        uint64_t cmax = chunks;
        for (auto &a : arms(e)) {
          std::string lab;
          for (uint32_t v : a.second) lab += "case " + u32(v) + ": ";
          line(lab + "{");
          ++ind;
          uint64_t ch = chunks;
          uint32_t wd = words;
          smax = std::max(smax, enc_block(a.first, end, slot, ch, wd, base, dadd));
          cmax = std::max(cmax, ch);
          wmax = std::max(wmax, wd);
          --ind;
          line("} break;");
        }
        if (e.flags & XDRG_F_DEFAULT) {
          line("default: {");
          ++ind;
          uint64_t ch = chunks;
          uint32_t wd = words;
          smax = std::max(smax, enc_block(e.arg4, end, slot, ch, wd, base, dadd));
          cmax = std::max(cmax, ch);
          wmax = std::max(wmax, wd);
          --ind;
          line("} break;");
        } else {
          line("default: return false;  // the size pass reported it");
        }
        line("}");
        --ind;
        line("}");
        slot = smax;
        chunks = cmax;
        words = wmax;
        pc = end;
        continue;
      }
      case XDRG_OP_VECTOR: {
        word_list = false;
        if (e.flags & XDRG_F_SUB) {  // each element walked by its body (payloads copied by the lane)
          const uint32_t k = uid++;
          const std::string ks = std::to_string(k);
          line("{");
          ++ind;
          line("const uint64_t eoff" + ks + " = *reinterpret_cast<const uint64_t *>(" + f + ");");
          line("const uint32_t cnt" + ks + " = ld32(" + f + " + 8);");
          line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
          line("c.put(bswap32(cnt" + ks + "));");
          // (unrolled as the size walk's, the encode measured slower: 84.1
          // vs 80.2 us, profiles/r05k)
          line("for (uint32_t i" + ks + " = 0; i" + ks + " < cnt" + ks + "; ++i" + ks + ") {");
          ++ind;
          const std::string el = load_elem(k, "(eoff" + ks + " + static_cast<uint64_t>(i" + ks + ") * " + u32(e.arg1) + ")",
                                            e.arg1, "c.heap", "c.heap_len");
          uint64_t ch = 0;
          uint32_t wd = 0;
          enc_block(e.arg4, body_end(e.arg4), kSlotMax, ch, wd, el, dadd + e.depth);
          --ind;
          line("}");
          --ind;
          line("}");
          ++pc;
          continue;
        }
        line("{");
        ++ind;
        line("const uint64_t eoff = *reinterpret_cast<const uint64_t *>(" + f + ");");
        line("const uint32_t cnt = ld32(" + f + " + 8);");
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line("c.put(bswap32(cnt));");
        line("uint32_t i = 0;");
        if (e.arg1 == 4 && e.arg2 == 1 && op(pc + 1).noff == 0 &&
            (op(pc + 1).kind == XDRG_OP_U32 || op(pc + 1).kind == XDRG_OP_ENUM || op(pc + 1).kind == XDRG_OP_BOOL)) {
          // 4-byte elements four at a time: one 16-byte load per four
          const xdrg_op &el = op(pc + 1);
          const std::string chk = "if (!c.field(" + u32(pc + 1) + ", " + depth(el, dadd) + ", 4)) return false;";
          auto cv = [&](const std::string &w) {
            return el.kind == XDRG_OP_BOOL ? "((" + w + " & 0xffu) ? 0x01000000u : 0u)" : "bswap32(" + w + ")";
          };
          line("for (; i + 4u <= cnt && eoff + 4ull * (i + 4u) <= c.heap_len; i += 4u) {");
          ++ind;
          line("const u32x4 t = ld16u(c.heap + eoff + 4ull * i);");
          for (const char *w : {"t.x", "t.y", "t.z", "t.w"}) line(chk + " c.put(" + cv(w) + ");");
          --ind;
          line("}");
        }
        line("for (; i < cnt; ++i) {");
        ++ind;
        line("const uint64_t eb = eoff + static_cast<uint64_t>(i) * " + u32(e.arg1) + ";");
        enc_elem(pc + 1, pc + 1 + e.arg2, e.arg1, dadd);
        --ind;
        line("}");
        --ind;
        line("}");
        pc += 1 + e.arg2;
        continue;
      }
      default: break;
      }
      ++pc;
    }
    return slot;
  }
  // Elements of a container (enc_vector_elems of xdrgpu.hip): fixed-size
  // fields read from the heap (bytes past heap_len read as 0).  An element
  // of 16-byte multiples whose word fields are 4-aligned is loaded whole
  // (16-byte loads) into registers first, its fields taken from there.
  bool enc_elem_regs(uint32_t b0, uint32_t b1, uint32_t es, uint32_t dadd) {
    if (es == 0 || (es & 15u) || es > 64) return false;
    for (uint32_t k = b0; k < b1; ++k) {
      const xdrg_op &e = op(k);
      if (e.kind != XDRG_OP_BOOL && (e.noff & 3u)) return false;
    }
    const uint32_t nw = es / 4;
    line("uint32_t ew[" + u32(nw) + "];");
    line("if (eb + " + u32(es) + " <= c.heap_len) {");
    for (uint32_t q = 0; q < nw; q += 4)
      line("  { const u32x4 t = ld16u(c.heap + eb + " + u32(4 * q) + "); ew[" + u32(q) + "] = t.x; ew[" +
           u32(q + 1) + "] = t.y; ew[" + u32(q + 2) + "] = t.z; ew[" + u32(q + 3) + "] = t.w; }");
    line("} else {");
    for (uint32_t q = 0; q < nw; ++q) line("  ew[" + u32(q) + "] = c.hword(eb + " + u32(4 * q) + ");");
    line("}");
    for (uint32_t k = b0; k < b1; ++k) {
      const xdrg_op &e = op(k);
      const std::string P = u32(k), D = depth(e, dadd), w = "ew[" + u32(e.noff / 4) + "]";
      line("if (!c.field(" + P + ", " + D + ", " + u32(4u * wire_words(e)) + ")) return false;");
      switch (e.kind) {
      case XDRG_OP_BOOL:
        line("c.put(((" + w + " >> " + std::to_string(8 * (e.noff % 4)) + ") & 0xffu) ? 0x01000000u : 0u);");
        break;
      case XDRG_OP_U64:
        line("c.put(bswap32(ew[" + u32(e.noff / 4 + 1) + "]));");
        line("c.put(bswap32(" + w + "));");
        break;
      case XDRG_OP_OPAQUE:
        for (uint32_t q = 0; 4 * q < e.arg0; ++q) {
          std::string x = "ew[" + u32(e.noff / 4 + q) + "]";
          if (4 * q + 4 > e.arg0) x = "(" + x + " & " + u32((1u << (8 * (e.arg0 - 4 * q))) - 1u) + ")";
          line("c.put(" + x + ");");
        }
        break;
      default: line("c.put(bswap32(" + w + "));"); break;
      }
    }
    return true;
  }
  void enc_elem(uint32_t b0, uint32_t b1, uint32_t es, uint32_t dadd) {
    if (enc_elem_regs(b0, b1, es, dadd)) return;
    for (uint32_t k = b0; k < b1; ++k) {
      const xdrg_op &e = op(k);
      const std::string P = u32(k), D = depth(e, dadd), a = "eb + " + u32(e.noff);
      const uint32_t wb = 4u * wire_words(e);
      line("if (!c.field(" + P + ", " + D + ", " + u32(e.kind == XDRG_OP_OPAQUE ? wb : wb) + ")) return false;");
      switch (e.kind) {
      case XDRG_OP_BOOL: line("c.put((c.hword(" + a + ") & 0xffu) ? 0x01000000u : 0u);"); break;
      case XDRG_OP_U64:
        line("c.put(bswap32(c.hword(" + a + " + 4)));");
        line("c.put(bswap32(c.hword(" + a + ")));");
        break;
      case XDRG_OP_OPAQUE:
        for (uint32_t w = 0; 4 * w < e.arg0; ++w) {
          std::string x = "c.hword(" + a + " + " + u32(4 * w) + ")";
          if (4 * w + 4 > e.arg0) x = "(" + x + " & " + u32((1u << (8 * (e.arg0 - 4 * w))) - 1u) + ")";
          line("c.put(" + x + ");");
        }
        break;
      default: line("c.put(bswap32(c.hword(" + a + ")));"); break;
      }
    }
  }

  // ---------------------------------------------------------------- decode
  // xdr_generic_get field by field (marshal.h:142-211).
  void dec_block(uint32_t pc, uint32_t stop, const std::string &base = "nat", uint32_t dadd = 0) {
    while (pc != stop) {
      const xdrg_op &e = op(pc);
      const std::string f = base + " + " + u32(e.noff), P = u32(pc), D = depth(e, dadd);
      switch (e.kind) {
      case XDRG_OP_END: return;
      case XDRG_OP_JUMP: pc = e.arg0; continue;
      case XDRG_OP_U32:
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line("st32(" + f + ", bswap32(c.word()));");
        break;
      case XDRG_OP_ENUM:
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        if (e.flags & XDRG_F_VALIDATE) {
          line("{");
          ++ind;
          line("const uint32_t v = bswap32(c.word());");
          line("st32(" + f + ", v);");
          line("if (!" + enum_test("v", e.arg0, e.arg1) + ") return c.fail(" + P + ", XDRG_ERR_INVALID_ENUM);");
          --ind;
          line("}");
        } else {
          line("st32(" + f + ", bswap32(c.word()));");
        }
        break;
      case XDRG_OP_BOOL:
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line(base + "[" + u32(e.noff) + "] = c.word() != 0u;");
        break;
      case XDRG_OP_U64:
        line("if (!c.field(" + P + ", " + D + ", 8)) return false;");
        line("st32(" + f + " + 4, bswap32(c.word()));");
        line("st32(" + f + ", bswap32(c.word()));");
        break;
      case XDRG_OP_OPAQUE: {
        const uint32_t L = e.arg0;
        line("if (!c.field(" + P + ", " + D + ", " + u32(L) + ")) return false;");
        line("{");
        ++ind;
        for (uint32_t k = 0; k < L; k += 4) {
          line("{ const uint32_t w = c.peek(c.p + " + u32(k) + ");");
          for (uint32_t b = 0; b < 4 && k + b < L; ++b)
            line("  " + base + "[" + u32(e.noff + k + b) + "] = uint8_t(w >> " + std::to_string(8 * b) + "); ");
          line("}");
        }
        if (L & 3u)
          line("if (c.peek(c.p + " + u32(L & ~3u) + ") & " + u32(~((1u << (8 * (L & 3u))) - 1u)) +
               ") return c.fail(" + P + ", XDRG_ERR_NONZERO_PAD);");
        line("c.p += " + u32((L + 3u) & ~3u) + ";");
        --ind;
        line("}");
        break;
      }
      case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING: {
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line("{");
        ++ind;
        line("const uint32_t len = bswap32(c.word());");
        line("if (len > c.b - c.p) return c.fail(" + P + ", XDRG_ERR_OVERFLOW_GET);");
        line("if (len > " + u32(e.arg0) + ") return c.fail(" + P + ", " +
             (e.kind == XDRG_OP_STRING ? "XDRG_ERR_XSTRING_BOUND" : "XDRG_ERR_XVECTOR_BOUND") + ");");
        line("if ((len & 3u) && (c.peek(c.p + (len & ~3u)) & ~keep_mask(len & 3u)))"
             " return c.fail(" + P + ", XDRG_ERR_NONZERO_PAD);");
        line("*reinterpret_cast<uint64_t *>(" + f + ") = c.p;  // the payload stays in the stream");
        line("st32(" + f + " + 8, len);");
        line("c.p += (static_cast<uint64_t>(len) + 3u) & ~3ull;");
        --ind;
        line("}");
        break;
      }
      case XDRG_OP_UNION: {
        const uint32_t end = ipdom[pc];
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line("{");
        ++ind;
        line("const uint32_t d = bswap32(c.word());");
        if (e.flags & XDRG_F_VALIDATE)
          line("if (!" + enum_test("d", e.arg0, e.arg1) + ") return c.fail(" + P + ", XDRG_ERR_INVALID_ENUM);");
        line("switch (d) {");
        for (auto &a : arms(e)) {
          std::string lab;
          for (uint32_t v : a.second) lab += "case " + u32(v) + ": ";
          line(lab + "{");
          ++ind;
          line("st32(" + f + ", d);");
          dec_block(a.first, end, base, dadd);
          --ind;
          line("} break;");
        }
        line("default: {");
        ++ind;
        if (e.flags & XDRG_F_DEFAULT) {
          line("st32(" + f + ", d);");
          dec_block(e.arg4, end, base, dadd);
        } else {
          line("return c.fail(" + P + ", XDRG_ERR_BAD_DISCRIMINANT);");
        }
        --ind;
        line("} break;");
        line("}");
        --ind;
        line("}");
        pc = end;
        continue;
      }
      case XDRG_OP_VECTOR: {
        if (e.flags & XDRG_F_SUB) {
          // the element array (zeroed) from the element area, then each
          // element by its body; an element that fails leaves 1 + its
          // index in the container's xdrg_bytes_ref.rsv (sub_kernels.h)
          const std::string ks = std::to_string(uid++);
          line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
          line("{");
          ++ind;
          line("const uint32_t cnt" + ks + " = bswap32(c.word());");
          line("if (cnt" + ks + " > " + u32(e.arg0) + ") return c.fail(" + P + ", " +
               ((e.flags & XDRG_F_POINTER) ? "XDRG_ERR_POINTER_BOUND" : "XDRG_ERR_XVECTOR_BOUND") + ");");
          line("if (!c.area_sub(" + P + ", cnt" + ks + ", " + u32(e.arg1) + ", " + u32(e.arg3) + ")) return false;");
          line("*reinterpret_cast<uint64_t *>(" + f + ") = c.ecur;");
          line("st32(" + f + " + 8, cnt" + ks + ");");
          line("uint8_t *arr" + ks + " = c.heap + c.ecur;");
          line("if (!c.zeroed)");
          line("  for (uint64_t z = 0; z < static_cast<uint64_t>(cnt" + ks + ") * " + u32(e.arg1) +
               "; z += 4) st32(arr" + ks + " + z, 0u);");
          line("c.ecur += static_cast<uint64_t>(cnt" + ks + ") * " + u32(e.arg1) + ";");
          line("for (uint32_t i" + ks + " = 0; i" + ks + " < cnt" + ks + "; ++i" + ks + ") {");
          ++ind;
          line("uint8_t *e" + ks + " = arr" + ks + " + static_cast<uint64_t>(i" + ks + ") * " + u32(e.arg1) + ";");
          line("auto body" + ks + " = [&]() -> bool {");
          ++ind;
          dec_block(e.arg4, body_end(e.arg4), "e" + ks, dadd + e.depth);
          line("return true;");
          --ind;
          line("};");
          line("if (!body" + ks + "()) { st32(" + f + " + 12, i" + ks + " + 1u); return false; }");
          --ind;
          line("}");
          --ind;
          line("}");
          ++pc;
          continue;
        }
        line("if (!c.field(" + P + ", " + D + ", 4)) return false;");
        line("{");
        ++ind;
        line("const uint32_t cnt = bswap32(c.word());");
        line("if (cnt > " + u32(e.arg0) + ") return c.fail(" + P + ", " +
             ((e.flags & XDRG_F_POINTER) ? "XDRG_ERR_POINTER_BOUND" : "XDRG_ERR_XVECTOR_BOUND") + ");");
        line("if (!c.area(" + P + ", cnt, " + u32(e.arg1) + ", " + u32(e.arg3) + ")) return false;");
        line("*reinterpret_cast<uint64_t *>(" + f + ") = c.ecur;");
        line("st32(" + f + " + 8, cnt);");
        line("uint32_t i = 0;");
        {
          const xdrg_op &el = op(pc + 1);
          if (e.arg1 == 4 && e.arg2 == 1 && el.noff == 0 &&
              (el.kind == XDRG_OP_U32 || el.kind == XDRG_OP_BOOL ||
               (el.kind == XDRG_OP_ENUM && !(el.flags & XDRG_F_VALIDATE)))) {
            // 4-byte elements two at a time: one 8-byte store per pair (the
            // array starts 8-aligned); a failing element leaves what the
            // one-by-one form leaves (the element before it stored, it zeroed)
            const std::string chk = "c.field(" + u32(pc + 1) + ", " + depth(el, dadd) + ", 4)";
            const std::string rsv = "st32(" + f + " + 12, ";
            auto cv = [&](const std::string &w) {
              return el.kind == XDRG_OP_BOOL ? "(" + w + " != 0u ? 1u : 0u)" : "bswap32(" + w + ")";
            };
            line("for (; i + 2u <= cnt; i += 2u) {");
            ++ind;
            line("uint8_t *ep = c.heap + c.ecur + 4ull * i;");
            line("if (!" + chk + ") { st32(ep, 0u); " + rsv + "i); return false; }");
            line("const uint32_t v0 = " + cv("c.word()") + ";");
            line("if (!" + chk + ") { st32(ep, v0); st32(ep + 4, 0u); " + rsv + "i + 1u); return false; }");
            line("const uint32_t v1 = " + cv("c.word()") + ";");
            line("*reinterpret_cast<unsigned long long *>(ep) = v0 | (static_cast<unsigned long long>(v1) << 32);");
            --ind;
            line("}");
          }
        }
        line("for (; i < cnt; ++i) {");
        ++ind;
        line("uint8_t *el = c.heap + c.ecur + static_cast<uint64_t>(i) * " + u32(e.arg1) + ";");
        dec_elem(pc, pc + 1, pc + 1 + e.arg2, e.arg1, base, dadd);
        --ind;
        line("}");
        line("c.ecur += static_cast<uint64_t>(cnt) * " + u32(e.arg1) + ";");
        --ind;
        line("}");
        pc += 1 + e.arg2;
        continue;
      }
      default: break;
      }
      ++pc;
    }
  }
  // One element of a container (dec_vector_elems of xdrgpu.hip): zero the
  // element, then its fields; an error in element i records i in the
  // container's xdrg_bytes_ref.rsv (the elements before it are decoded).
  // Elements of up to 64 bytes whose word fields are 4-aligned are built in
  // registers and leave as whole 8- or 4-byte stores (a lane's scattered
  // byte and word stores were most of vecrec's decode); a failing field
  // stores what was built so far, as the store-by-store form leaves it.
  bool dec_elem_regs(uint32_t vpc, uint32_t b0, uint32_t b1, uint32_t es, const std::string &base, uint32_t dadd) {
    if ((es & 3u) || es == 0 || es > 64) return false;
    for (uint32_t k = b0; k < b1; ++k) {
      const xdrg_op &e = op(k);
      if (e.kind != XDRG_OP_BOOL && e.kind != XDRG_OP_OPAQUE && (e.noff & 3u)) return false;
    }
    const uint32_t nw = es / 4;
    std::string store;
    if ((es & 7u) == 0) {
      for (uint32_t z = 0; z < nw; z += 2)
        store += "*reinterpret_cast<unsigned long long *>(el + " + u32(4 * z) + ") = ew[" + u32(z) +
                 "] | (static_cast<unsigned long long>(ew[" + u32(z + 1) + "]) << 32); ";
    } else {
      for (uint32_t z = 0; z < nw; ++z) store += "st32(el + " + u32(4 * z) + ", ew[" + u32(z) + "]); ";
    }
    const std::string fail_done = store + "st32(" + base + " + " + u32(op(vpc).noff) + " + 12, i); ";
    line("uint32_t ew[" + u32(nw) + "] = {};");
    auto byte_in = [&](uint32_t at, const std::string &v) {
      return "ew[" + u32(at / 4) + "] |= (" + v + ") << " + std::to_string(8 * (at % 4)) + ";";
    };
    for (uint32_t k = b0; k < b1; ++k) {
      const xdrg_op &e = op(k);
      const std::string P = u32(k), D = depth(e, dadd);
      const uint32_t need = e.kind == XDRG_OP_U64 ? 8u : e.kind == XDRG_OP_OPAQUE ? e.arg0 : 4u;
      line("if (!c.field(" + P + ", " + D + ", " + u32(need) + ")) { " + fail_done + "return false; }");
      switch (e.kind) {
      case XDRG_OP_BOOL: line(byte_in(e.noff, "c.word() != 0u ? 1u : 0u")); break;
      case XDRG_OP_U64:
        line("{ const uint32_t hi = bswap32(c.word()), lo = bswap32(c.word());");
        line("  ew[" + u32(e.noff / 4) + "] = lo; ew[" + u32(e.noff / 4 + 1) + "] = hi; }");
        break;
      case XDRG_OP_OPAQUE: {
        const uint32_t L = e.arg0;
        for (uint32_t q = 0; q < L; q += 4) {
          line("{ const uint32_t w = c.peek(c.p + " + u32(q) + ");");
          for (uint32_t b = 0; b < 4 && q + b < L; ++b)
            line("  " + byte_in(e.noff + q + b, "(w >> " + std::to_string(8 * b) + ") & 0xffu"));
          line("}");
        }
        if (L & 3u)
          line("if (c.peek(c.p + " + u32(L & ~3u) + ") & " + u32(~((1u << (8 * (L & 3u))) - 1u)) + ") { " +
               fail_done + "return c.fail(" + P + ", XDRG_ERR_NONZERO_PAD); }");
        line("c.p += " + u32((L + 3u) & ~3u) + ";");
        break;
      }
      default: {
        line("{ const uint32_t v = bswap32(c.word());");
        line("  ew[" + u32(e.noff / 4) + "] = v;");
        if (e.kind == XDRG_OP_ENUM && (e.flags & XDRG_F_VALIDATE))
          line("  if (!" + enum_test("v", e.arg0, e.arg1) + ") { " + fail_done + "return c.fail(" + P +
               ", XDRG_ERR_INVALID_ENUM); }");
        line("}");
        break;
      }
      }
    }
    line(store);
    return true;
  }
  void dec_elem(uint32_t vpc, uint32_t b0, uint32_t b1, uint32_t es, const std::string &base, uint32_t dadd) {
    if (dec_elem_regs(vpc, b0, b1, es, base, dadd)) return;
    const std::string fail_done = "st32(" + base + " + " + u32(op(vpc).noff) + " + 12, i); ";
    const bool w4 = (es & 3u) == 0;  // 4-byte stores (element arrays are 8-aligned)
    line("if (!c.zeroed) {");  // (the group's LDS stage is zeroed whole)
    if (w4)
      for (uint32_t z = 0; z < es; z += 4) line("  st32(el + " + u32(z) + ", 0u);");
    else
      line("  for (uint32_t z = 0; z < " + u32(es) + "; ++z) el[z] = 0;");
    line("}");
    for (uint32_t k = b0; k < b1; ++k) {
      const xdrg_op &e = op(k);
      const std::string P = u32(k), D = depth(e, dadd), f = "el + " + u32(e.noff);
      const uint32_t need = e.kind == XDRG_OP_U64 ? 8u : e.kind == XDRG_OP_OPAQUE ? e.arg0 : 4u;
      line("if (!c.field(" + P + ", " + D + ", " + u32(need) + ")) { " + fail_done + "return false; }");
      switch (e.kind) {
      case XDRG_OP_BOOL: line("el[" + u32(e.noff) + "] = c.word() != 0u;"); break;
      case XDRG_OP_U64:
        line("{ const uint32_t hi = bswap32(c.word()), lo = bswap32(c.word());");
        if (w4 && !(e.noff & 3u)) {
          line("  st32(" + f + ", lo); st32(" + f + " + 4, hi);");
        } else {
          for (int q = 0; q < 4; ++q)
            line("  el[" + u32(e.noff + q) + "] = uint8_t(lo >> " + std::to_string(8 * q) + "); el[" +
                 u32(e.noff + 4 + q) + "] = uint8_t(hi >> " + std::to_string(8 * q) + ");");
        }
        line("}");
        break;
      case XDRG_OP_OPAQUE: {
        const uint32_t L = e.arg0;
        for (uint32_t q = 0; q < L; q += 4) {
          line("{ const uint32_t w = c.peek(c.p + " + u32(q) + ");");
          for (uint32_t b = 0; b < 4 && q + b < L; ++b)
            line("  el[" + u32(e.noff + q + b) + "] = uint8_t(w >> " + std::to_string(8 * b) + ");");
          line("}");
        }
        if (L & 3u)
          line("if (c.peek(c.p + " + u32(L & ~3u) + ") & " + u32(~((1u << (8 * (L & 3u))) - 1u)) + ") { " +
               fail_done + "return c.fail(" + P + ", XDRG_ERR_NONZERO_PAD); }");
        line("c.p += " + u32((L + 3u) & ~3u) + ";");
        break;
      }
      default: {
        line("{ const uint32_t v = bswap32(c.word());");
        if (w4 && !(e.noff & 3u))
          line("  st32(" + f + ", v);");
        else
          line("  for (int q = 0; q < 4; ++q) el[" + u32(e.noff) + " + q] = uint8_t(v >> (8 * q));");
        if (e.kind == XDRG_OP_ENUM && (e.flags & XDRG_F_VALIDATE))
          line("  if (!" + enum_test("v", e.arg0, e.arg1) + ") { " + fail_done + "return c.fail(" + P +
               ", XDRG_ERR_INVALID_ENUM); }");
        line("}");
        break;
      }
      }
    }
  }
};

// A plan the generator handles: every construct of the op set, with the
// unions' post-dominators defined and inside the plan.
// Element subroutines are emitted inline per element: none may be entered
// from itself (recursive types run the frame walk, sub_kernels.h), and
// their elements (read into registers, load_elem) are at most 64 bytes.
bool supported(const gen &g) {
  for (uint32_t i = 0; i < g.nops(); ++i) {
    const xdrg_op &o = g.op(i);
    if (o.kind == XDRG_OP_UNION && (g.ipdom[i] == kNoPc || g.ipdom[i] >= g.nops())) return false;
    if (o.kind == XDRG_OP_VECTOR && (o.flags & XDRG_F_SUB) &&
        (o.arg1 == 0 || o.arg1 > 64 || (o.arg1 & 3u) || o.arg4 >= g.nops() || o.arg3 == 0))
      return false;
  }
  return true;
}

}  // namespace

namespace {
// Source hash line (xdrg_spec_src_hash, checked at module load) and the
// finished source.
void seal(std::string src, spec_info &info) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a
  for (unsigned char ch : src) h = (h ^ ch) * 1099511628211ull;
  info.src_hash = h;
  src += "extern \"C\" __device__ __attribute__((used)) unsigned long long xdrg_spec_src_hash = " +
         std::to_string(h) + "ull;\n";
  info.source = std::move(src);
}

// The record-start parse of the plain-stream index (plan_rx) and its index
// kernels: the list ranking's segment parse, the speculative walk over
// records up to the index window, the same walk over records of any length
// (xdrg_index_records with max_rec_len past the window: a record past the
// staged stretch parsed by the wave through blocks of the stream) and the
// one-wave repair of its failed segments (rxs_fix).
std::string rx_source(const std::string &first, const std::string &flen, const std::string &second,
                      const std::string &rx_code, const std::string &rxs_code) {
  std::ostringstream s;
  s << "struct plan_rx {  // index_kernels.h ix_seg_body's, rxs_walk_body's and rxs_fix_body's parser\n"
    << "  __device__ __forceinline__ void init(uint32_t *) const {}\n"
    << "  __device__ __forceinline__ bool first_ok(const uint32_t *, uint32_t v) const { return " << first << "; }\n"
    << "  __device__ __forceinline__ uint64_t first_len(uint32_t v) const { return " << flen << "; }\n"
    << "  __device__ __forceinline__ bool second_ok(uint32_t v, uint32_t w) const { return " << second << "; }\n"
    << "  __device__ __forceinline__ uint32_t rlen(const uint32_t *m, const uint8_t *__restrict__ s, uint64_t len,\n"
    << "                                           uint64_t a, uint32_t maxlen) const {\n"
    << "    return rlen_rd<rx_global, uint64_t>(m, rx_global{s}, len, a, maxlen);\n  }\n"
    << "  // U: the position type (uint32_t for offsets into a staged stretch)\n"
    << "  template <class RD, class U>\n"
    << "  __device__ __forceinline__ uint32_t rlen_rd(const uint32_t *, const RD &rd, U len,\n"
    << "                                              U a, uint32_t maxlen) const {\n"
    << "    const bool capped = static_cast<uint64_t>(a) + maxlen < len;\n"
    << "    [[maybe_unused]] const bool whole = maxlen > XDRG_INDEX_MAX_MSG;  // (tail lists: no frame bound)\n"
    << "    U lim = capped ? static_cast<U>(a + maxlen) : len;\n"
    << "    uint32_t past = capped ? RX_LONG : RX_BAD;\n"
    << "    rd.clamp(lim, past, a);  // (the staged stretch's end: RX_OUT, and the caller parses from global memory)\n"
    << "    U p = a;\n"
    << rx_code << "    return static_cast<uint32_t>(p - a);\n  }\n"
    << "  // the same parse over the staged stretch without early returns (index_kernels.h rxs_rlen)\n"
    << "  __device__ __forceinline__ uint32_t rlen_st(const uint32_t *, const rx_lds &rd, uint32_t len,\n"
    << "                                              uint32_t a, uint32_t maxlen) const {\n"
    << "    using U = uint32_t;\n"
    << "    const bool capped = static_cast<uint64_t>(a) + maxlen < len;\n"
    << "    [[maybe_unused]] const bool whole = maxlen > XDRG_INDEX_MAX_MSG;\n"
    << "    U lim = capped ? static_cast<U>(a + maxlen) : len;\n"
    << "    uint32_t past = capped ? RX_LONG : RX_BAD;\n"
    << "    rd.clamp(lim, past, a);\n"
    << "    uint32_t r = 0;\n"
    << "    U p = a;\n"
    << rxs_code << "    return r ? r : static_cast<uint32_t>(p - a);\n  }\n"
    << "};\n\n"
    << "extern \"C\" __global__ __launch_bounds__(256) void xdrg_spec_ix_seg(\n"
    << "    const uint8_t *s, uint64_t len, uint32_t maxlen, uint32_t K, uint64_t *tab, uint32_t *list,\n"
    << "    uint32_t *lcount, uint32_t has_first, uint32_t fd, const uint32_t *skip) {\n"
    << "  if (skip && *skip == 1u) return;  // the speculative walk holds the index\n"
    << "  ix_seg_body<true>(plan_rx{}, s, len, maxlen, K, tab, list, lcount, has_first != 0, fd);\n}\n\n"
    << "extern \"C\" __global__ __launch_bounds__(64) void xdrg_spec_rxs_walk(\n"
    << "    const uint8_t *s, uint64_t len, uint32_t maxlen, uint64_t *seg, uint16_t *nodes,\n"
    << "    uint32_t *flag, uint32_t has_first, uint32_t fd) {\n"
    << "  rxs_walk_body(plan_rx{}, s, len, maxlen, seg, nodes, flag, has_first != 0, fd);\n}\n\n"
    << "extern \"C\" __global__ __launch_bounds__(64) void xdrg_spec_rxs_walk_whole(\n"
    << "    const uint8_t *s, uint64_t len, uint32_t maxlen, uint64_t *seg, uint16_t *nodes,\n"
    << "    uint32_t *flag, uint32_t has_first, uint32_t fd) {\n"
    << "  rxs_walk_body<true>(plan_rx{}, s, len, maxlen, seg, nodes, flag, has_first != 0, fd);\n}\n\n"
    << "extern \"C\" __global__ __launch_bounds__(64) void xdrg_spec_rxs_fix(\n"
    << "    const uint8_t *s, uint64_t len, uint32_t maxlen, uint64_t *seg, uint64_t nseg, uint16_t *nodes,\n"
    << "    const uint64_t *list, const unsigned long long *nl, uint32_t *flag, unsigned long long *cnt) {\n"
    << "  rxs_fix_body(plan_rx{}, s, len, maxlen, seg, nseg, nodes, list, nl, flag, cnt);\n}\n\n";
  return s.str();
}

// A recursive plan whose recursion is a linked list: the record's last
// field is a pointer (count 0 or 1) to another record of the same plan,
// and nothing before it holds element subroutines (rpcbind's rp__list,
// xdrpp/rpcb_prot.x:32-37).  Its record parse is a loop over the list's
// nodes (vpc: the pointer's op).
bool tail_list(const gen &g, uint32_t &vpc) {
  uint32_t end = 0;
  while (end < g.nops() && g.op(end).kind != XDRG_OP_END) ++end;
  if (end == 0 || end >= g.nops()) return false;
  vpc = end - 1;
  const xdrg_op &v = g.op(vpc);
  if (v.kind != XDRG_OP_VECTOR || !(v.flags & XDRG_F_SUB) || v.arg4 != 0 || v.arg0 != 1) return false;
  for (uint32_t pc = 0; pc < vpc; ++pc) {
    const xdrg_op &o = g.op(pc);
    if (o.kind == XDRG_OP_VECTOR && (o.flags & XDRG_F_SUB)) return false;
    if (o.kind == XDRG_OP_JUMP && o.arg0 > vpc) return false;
    if (o.kind == XDRG_OP_UNION && (g.ipdom[pc] == kNoPc || g.ipdom[pc] > vpc)) return false;
  }
  return true;
}

// The tail list's parse: the node's fields, then the pointer's count, node
// after node.  xdro_index_records' rx_walk (oracle/xdr_oracle.c) opens a
// frame per node in the index window (past XDRG_INDEX_FRAMES: RX_LONG) and
// lets a tail pointer's node take its parent's frame in the whole-record
// walk (whole: max_rec_len past the window), so there the list has no bound.
std::string tail_rx(gen &g, uint32_t vpc, bool sticky) {
  g.o.str("");
  g.ind = 6;
  g.rx_sticky = sticky;
  g.rx_block(0, vpc);
  g.rx_sticky = false;
  const std::string body = g.o.str();
  std::ostringstream s;
  if (!sticky) {
    s << "    for (uint32_t fr = 0;; ++fr) {  // a node of the list\n" << body
      << "      if (lim - p < 4u) return past;\n"
      << "      const uint32_t v = bswap32(rd.at(p));\n"
      << "      p += 4u;\n"
      << "      if (v > 1u) return RX_BAD;\n"
      << "      if (!v) break;\n"
      << "      if (!whole && fr == XDRG_INDEX_FRAMES) return RX_LONG;\n"
      << "    }\n";
  } else {
    s << "    for (uint32_t fr = 0; r == 0u; ++fr) {  // a node of the list\n" << body
      << "      r = (r == 0u && (lim - p < 4u)) ? past : r;\n"
      << "      const uint32_t v = bswap32(rd.atc(p));\n"
      << "      p += 4u;\n"
      << "      r = (r == 0u && (v > 1u)) ? RX_BAD : r;\n"
      << "      if (!v) break;\n"
      << "      r = (r == 0u && !whole && fr == XDRG_INDEX_FRAMES) ? RX_LONG : r;\n"
      << "    }\n";
  }
  return s.str();
}

// Recursive plans (element subroutines entered from themselves: rp__list,
// test_recursive): the frame walks of sub_kernels.h over this plan's ops as
// compile-time constants.  plan_ops::visit switches on the walk's pc; an op
// that always continues at the next one (a scalar field) falls through to
// it, so a struct's run of fields is one dispatch, not one per field.
// The element image a generated frame walk keeps in registers
// (sub_kernels.h sub_src_t): the largest element subroutine's stride, in
// whole 16-byte loads, at most kMaxImgWords words.
uint32_t img_words(const xdrg_plan &p) {
  uint32_t b = 0;
  for (const xdrg_op &o : p.ops)
    if (o.kind == XDRG_OP_VECTOR && (o.flags & XDRG_F_SUB)) b = std::max(b, o.arg1);
  return std::min((b + 15u) / 16u * 4u, kMaxImgWords);
}

bool frame_walk_source(const xdrg_plan &p, spec_info &info) {
  std::ostringstream s;
  s << "// Generated by libxdrgpu (codegen.cpp) from a recursive plan of " << p.ops.size()
    << " ops: the frame walks of sub_kernels.h with the ops as constants.\n"
    << "#include \"sub_kernels.h\"\n"
    << "#include \"index_kernels.h\"\n"
    << "using namespace xdrg::dev;\n\n"
    << "extern \"C\" __device__ __attribute__((used)) unsigned xdrg_spec_iface = " << kSpecIface << "u;\n\n"
    << "struct plan_ops {\n"
    << "  static constexpr uint32_t kImgWords = " << img_words(p) << "u;\n"
    << "  template <class F>\n"
    << "  __device__ __forceinline__ static int visit(const xdrg_op *, uint32_t &pc, F &&step) {\n"
    << "    int rc;\n"
    << "    switch (pc) {\n";
  const uint32_t n = static_cast<uint32_t>(p.ops.size());
  for (uint32_t i = 0; i < n; ++i) {
    const xdrg_op &o = p.ops[i];
    const bool seq = o.kind == XDRG_OP_U32 || o.kind == XDRG_OP_U64 || o.kind == XDRG_OP_BOOL ||
                     o.kind == XDRG_OP_ENUM || o.kind == XDRG_OP_OPAQUE || o.kind == XDRG_OP_VAROPAQUE ||
                     o.kind == XDRG_OP_STRING;
    std::ostringstream t;
    t << "step(xop<" << unsigned(o.kind) << "u, " << unsigned(o.flags) << "u, " << unsigned(o.depth) << "u, "
      << o.noff << "u, " << o.arg0 << "u, " << o.arg1 << "u, " << o.arg2 << "u, " << o.arg3 << "u, " << o.arg4
      << "u>{})";
    s << "    case " << i << "u:";
    if (seq && i + 1 < n)
      s << " rc = " << t.str() << "; if (rc != kWalkCont || pc != " << i + 1 << "u) return rc; [[fallthrough]];\n";
    else
      s << " return " << t.str() << ";\n";
  }
  s << "    default: return kWalkErr;\n"
    << "    }\n  }\n};\n\n"
    << "extern \"C\" __global__ __launch_bounds__(256) void xdrg_spec_sub_size(XDRG_SUB_SIZE_PARAMS) {\n"
    << "  sub_size_kernel<false, plan_ops>(XDRG_SUB_SIZE_ARGS);\n}\n"
    << "extern \"C\" __global__ __launch_bounds__(256) void xdrg_spec_sub_depth(XDRG_SUB_SIZE_PARAMS) {\n"
    << "  sub_size_kernel<true, plan_ops>(XDRG_SUB_SIZE_ARGS);\n}\n"
    << "extern \"C\" __global__ __launch_bounds__(256) void xdrg_spec_sub_encode(XDRG_SUB_ENCODE_PARAMS) {\n"
    << "  sub_encode_kernel<plan_ops>(XDRG_SUB_ENCODE_ARGS);\n}\n"
    << "extern \"C\" __global__ __launch_bounds__(256) void xdrg_spec_sub_decode(XDRG_SUB_DECODE_PARAMS) {\n"
    << "  sub_decode_kernel<plan_ops>(XDRG_SUB_DECODE_ARGS);\n}\n"
    << "extern \"C\" __global__ __launch_bounds__(256) void xdrg_spec_sub_chain(XDRG_SUB_ENCODE_PARAMS) {\n"
    << "  sub_chain_kernel<plan_ops>(XDRG_SUB_ENCODE_ARGS);\n}\n"
    << "extern \"C\" __global__ __launch_bounds__(256) void xdrg_spec_sub_chain_size(XDRG_SUB_SIZE_PARAMS) {\n"
    << "  sub_chain_size_kernel<plan_ops>(XDRG_SUB_SIZE_ARGS);\n}\n\n";
  info = spec_info{};
  info.frame_walk = true;
  gen g(p);
  uint32_t vpc = 0;
  if (tail_list(g, vpc)) {  // the index's record parse, a loop over the list's nodes
    const std::string rx_code = tail_rx(g, vpc, false), rxs_code = tail_rx(g, vpc, true);
    s << rx_source(g.first_test(), g.first_len(), g.second_test(), rx_code, rxs_code);
    info.tail_rx = true;
  }
  seal(s.str(), info);
  return true;
}
}  // namespace

bool spec_source(const xdrg_plan &p, spec_info &info) {
  if (p.path != XDRG_PATH_VAR) return false;
  if (p.deep) return frame_walk_source(p, info);  // recursive / deep nesting: the frame walk
  gen g(p);
  if (!supported(g)) return false;
  std::ostringstream body;
  // size
  g.o.str("");
  g.ind = 2;
  g.size_block(0, kNoPc, "nat");
  const std::string size_code = g.o.str();
  // encode
  g.o.str("");
  g.ind = 2;
  uint64_t chunks = 0;
  uint32_t words = 0;
  const uint32_t slots = g.enc_block(0, kNoPc, 0, chunks, words);
  // the word list (mark + words, 4 bytes each per lane) must fit in the
  // tile it aliases, and the walk must run from registers
  const bool regs = p.stride <= kRegRecordBytes && p.stride % 4 == 0;
  const uint32_t kwords = g.word_list && regs && words + 1 <= kMaxListWords && 4 * (words + 1) <= p.stride ? words : 0;
  const std::string enc_code = g.o.str();
  // decode
  g.o.str("");
  g.ind = 2;
  g.dec_block(0, kNoPc);
  const std::string dec_code = g.o.str();
  // record parse of the plain-stream index
  g.o.str("");
  g.ind = 2;
  g.rx_block(0, kNoPc);
  const std::string rx_code = g.o.str();
  g.o.str("");
  g.rx_sticky = true;
  g.rx_block(0, kNoPc);
  g.rx_sticky = false;
  const std::string rxs_code = g.o.str();
  const std::string first = g.first_test(), flen = g.first_len(), second = g.second_test();
  // element-area shares of packed plans
  g.o.str("");
  g.ind = 4;
  if (p.packed) g.eb_block(0, kNoPc, true);
  const std::string eb_code = g.o.str();

  const uint32_t maxd = g.maxd;  // deepest field: the stack budget a wave must have to skip the checks
  info.slots = std::max<uint32_t>(1, slots);
  info.dec_regs = regs;
  info.word_list = kwords > 0;
  info.list_words = kwords > 0 ? kwords + 1 : 0;
  info.max_chunks = chunks;
  std::ostringstream s;
  s << "// Generated by libxdrgpu (codegen.cpp) from a plan of " << p.ops.size()
    << " ops: straight-line walker for var_kernels.h.\n"
    << "#include \"var_kernels.h\"\n"
    << "#include \"index_kernels.h\"\n"
    << "using namespace xdrg::dev;\n\n"
    << "extern \"C\" __device__ __attribute__((used)) unsigned xdrg_spec_iface = " << kSpecIface << "u;\n\n"
    << "struct plan_walk {\n"
    << "  __device__ __forceinline__ uint64_t size(const uint8_t *nat, const uint8_t *heap, uint64_t heap_len,\n"
    << "                                             uint32_t &bad_op) const {\n"
    << "    uint64_t s = 0;\n"
    << size_code << "    return s;\n  }\n"
    << "  static constexpr bool kFastWalk = true;  // enc() also runs on an unchecked context\n"
    << "  static constexpr bool kDirect = true;    // ... and on var_kernels.h enc_direct_ctx\n"
    << "  static constexpr uint32_t kMaxDepth = " << maxd << "u;\n"
    << "  static constexpr uint32_t kWords = " << kwords << "u;  // scalar words per record (0: no word list)\n"
    << "  template <class CTX>\n"
    << "  __device__ __forceinline__ bool enc(CTX &c, const uint8_t *nat, bool ok) const {\n"
    << "    if (!ok) return false;\n"
    << enc_code << "    return true;\n  }\n"
    << "  template <bool RA>\n"
    << "  __device__ __forceinline__ bool dec(dec_ctx<RA> &c, uint8_t *nat, bool ok) const {\n"
    << "    if (!ok) return false;\n"
    << dec_code << "    return true;\n  }\n"
    << "  __device__ __forceinline__ bool packed() const { return " << (p.packed ? "true" : "false") << "; }\n"
    << "  template <class RD>\n"
    << "  __device__ __forceinline__ uint64_t ebytes(RD &rd, uint64_t q, uint64_t b, bool on) const {\n"
    << "    uint64_t E = 0;\n"
    << "    if (!on) return E;\n"
    << "    {\n" << eb_code << "    }\n"
    << "    return E;\n  }\n"
    << "};\n\n"
    << rx_source(first, flen, second, rx_code, rxs_code)
    << "extern \"C\" __global__ __launch_bounds__(64) void xdrg_spec_size(\n"
    << "    const uint8_t *native, uint64_t n, uint32_t stride, const uint8_t *heap, uint64_t heap_len,\n"
    << "    uint32_t *sizes, unsigned long long *block_sums, uint32_t mark, unsigned long long *err) {\n"
    << "  var_size_body<plan_walk, " << (regs ? p.stride / 4 : 0)
    << ">(plan_walk{}, native, n, stride, heap, heap_len, sizes, block_sums, mark, err);\n}\n\n"
    << "extern \"C\" __global__ __launch_bounds__(64) void xdrg_spec_encode(\n"
    << "    const uint8_t *native, uint64_t n, uint32_t stride, const uint8_t *heap, uint64_t heap_len,\n"
    << "    uint8_t *xdr, uint64_t cap, uint64_t *offsets, const uint32_t *sizes,\n"
    << "    const unsigned long long *block_base, uint32_t stack_limit, uint32_t C,\n"
    << "    uint32_t mark, unsigned long long *err) {\n"
    << "  var_encode_body<plan_walk, " << info.slots << ", 4, " << (regs ? p.stride / 4 : 0) << ", "
    << (kwords > 0 ? 4096 : 8192) << "u>(plan_walk{}, native, n, stride, heap, heap_len,\n"
    << "      xdr, cap, offsets, sizes, block_base, stack_limit, C, mark, err);\n}\n\n";
  // word-list plans: the encode walked first -- the wave's base by a
  // look-back (no size pass, no scan), or from xdrg_encode_sizes' scan
  if (kwords > 0)
    for (int lb = 0; lb < 2; ++lb)
      s << "extern \"C\" __global__ __launch_bounds__(64, XDRG_PRE_WAVES) void xdrg_spec_encode_" << (lb ? "lb" : "pre") << "(\n"
        << "    const uint8_t *native, uint64_t n, uint32_t stride, const uint8_t *heap, uint64_t heap_len,\n"
        << "    uint8_t *xdr, uint64_t cap, uint64_t *offsets, const unsigned long long *block_base,\n"
        << "    unsigned long long *desc, uint32_t nb, uint64_t *total, uint32_t stack_limit, uint32_t C,\n"
        << "    uint32_t mark, unsigned long long *err) {\n"
        << "  var_encode_body<plan_walk, " << info.slots << ", 4, " << p.stride / 4 << ", 4096u, " << (lb ? 1 : 2)
        << ">(plan_walk{}, native, n, stride, heap, heap_len,\n"
        << "      xdr, cap, offsets, nullptr, block_base, stack_limit, C, mark, err, desc, nb, total);\n}\n\n";
  for (int cp = 0; cp < 2; ++cp)
    s << "extern \"C\" __global__ __launch_bounds__(64) void xdrg_spec_decode" << (cp ? "_copy" : "") << "(\n"
      << "    const uint8_t *xdr, uint64_t len, const uint64_t *offsets, uint64_t n, uint8_t *native,\n"
      << "    uint32_t stride, uint8_t *heap, uint32_t stack_limit, uint32_t C, uint64_t ebase,\n"
      << "    uint32_t F, uint32_t mark, uint32_t S, unsigned long long *err) {\n"
      << "  var_decode_body<plan_walk, " << (cp ? "true" : "false")
      << ", true, " << (regs ? p.stride / 4 : 0) << ">(plan_walk{}, xdr, len, offsets, n, native, stride, heap,\n"
      << "      stack_limit, C, ebase, F, mark, S, err);\n}\n\n";
  // the source's own hash, defined in it: spec_get refuses a code object
  // (kernel cache file, or one attached with xdrg_plan_load_kernels) that
  // was not compiled from this plan's source
  seal(s.str(), info);
  return true;
}

}  // namespace xdrg
