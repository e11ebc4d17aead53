// xdrc back end: device plans at generation time.
//
// gen_hh (xdrc/gen_hh.cc:817-899) walks xdrc's symlist and writes the C++
// types with their xdr_traits<T>::save/load.  gen_plan walks the same
// symlist (xdrc/xdrc_internal.h) and writes, for every struct and union
// (and typedef naming one), the plan xdrg_plan_create takes: the wire-ordered
// op table, the case/enum table, the staged native stride, the fixed wire
// size, the bad-discriminant what() of each union op (gen_hh.cc:479-481), a
// C create function, and -- when the types xdrc -hh emitted are visible --
// a C++ xdr::gpu::emitted_plan<T> specialization that include/xdrpp_gpu.hh
// takes instead of recording the plan from xdr_traits<T> at run time.  With
// `-kernels DIR` it also writes each variable-length type's specialized
// kernel source (xdrg_plan_kernel_source, host-only) for hipcc --genco at
// build time; the emitted plan names the code object, so nothing is
// recorded or compiled at run time.
//
// The plan of a type is what xdr_generic_put/get walk (marshal.h:84-211)
// through xdr_traits: struct fields in order (gen_hh.cc:212-250), a union's
// discriminant then the selected arm (gen_hh.cc:575-675), containers as a
// count then their elements (types.h:374-392, :476-512, :591-665).  Layout
// and op conventions are the library's (include/xdrgpu.h); the op list is
// identical, op for op, to what xdrpp_amd/xdr_types.py compiles and what
// xdr::gpu::plan_for<T>() records (tests/test_gen_plan.py,
// tests/cpp/emitted_test.cc).
//
// Entry point: gen_plan(std::ostream &, const plan_gen_options &), called by
// xdrc's driver for `xdrc -plan` (here oracle/xdrc_driver.cc).
#include "xdrc/xdrc_internal.h"  // xdrc's AST (symlist)
#include "gen_plan.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <stdexcept>

#include "xdrgpu.h"

namespace xdrg_gen {
namespace {

constexpr uint32_t kMaxLen = 0xfffffffcu;  // XDR_MAX_LEN (xdrpp/types.h:360), the bound of x<>

uint32_t align_up(uint32_t x, uint32_t a) { return (x + a - 1) / a * a; }

std::string local_name(const std::string &n) {
  const size_t k = n.rfind("::");
  return k == std::string::npos ? n : n.substr(k + 2);
}

std::string c_ident(const std::string &n) {
  std::string s;
  for (unsigned char c : n) s += std::isalnum(c) || c == '_' ? static_cast<char>(c) : '_';
  return s;
}

// ------------------------------------------------------------ resolved types
enum class kind { scalar, enm, opaque_array, varbytes, xarray, xvector, strct, unn, vd, unsupported };

struct type_t;
struct field_t {
  std::string name;
  type_t *t;
  uint32_t off;
};
struct arm_t {
  std::vector<uint32_t> cases;
  std::string name;
  type_t *t;  // the void type for a void arm
};

struct type_t {
  kind k = kind::scalar;
  std::string name;     // struct / union / enum id (xdrc's, anonymous ones as _<field>_t)
  std::string cxx;      // C++ qualified name of a top-level struct/union ("" otherwise)
  uint8_t op = 0;       // scalar: XDRG_OP_U32 / U64 / BOOL; varbytes: VAROPAQUE / STRING
  uint32_t size = 0, align = 1;
  bool fixed = false;   // xdr_traits<T>::fixed_size
  uint64_t wire = 0;    // fixed wire bytes
  uint32_t n = 0;       // opaque[n], T x[n], max length of x<n> / opaque<n> / string<n>
  type_t *elem = nullptr;
  bool pointer = false;
  std::vector<uint32_t> enum_vals;  // sorted distinct tag values
  bool validate = false;            // enum opting in to xdr_validate_enum (types.h:157-173)
  std::vector<field_t> fields;
  std::string tag_name;
  type_t *tag = nullptr;
  std::vector<arm_t> arms;
  bool has_default = false;
  arm_t def;
  uint32_t arms_off = 0;
  std::string why;  // unsupported: the reason
  std::vector<std::string> enums_cxx;  // C++ names of enums reachable (validation checks)
};

struct gen_error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------ plan builder
// The wire-ordered flattening of a type: the record's ops, END, then one
// element subroutine per element type that is not fixed-size, breadth first
// in order of first reference (the order xdr_types.py and the C++ recorder
// use), each ending with END.
struct plan_ctx {
  std::vector<xdrg_op> ops;
  std::vector<uint32_t> table;
  std::map<uint32_t, std::string> msgs;  // op -> bad-discriminant what()
  struct sub { type_t *t; uint32_t entry; std::vector<uint32_t> vecs; };
  std::vector<sub> subs;
  std::deque<size_t> pending;

  uint32_t emit(uint8_t k, uint32_t noff, uint32_t depth, uint8_t flags = 0, uint32_t a0 = 0, uint32_t a1 = 0,
                uint32_t a2 = 0, uint32_t a3 = 0, uint32_t a4 = 0) {
    if (depth > 0xffffu) throw gen_error("nesting deeper than 65535 levels");
    xdrg_op o{};
    o.kind = k;
    o.flags = flags;
    o.depth = static_cast<uint16_t>(depth);
    o.noff = noff;
    o.arg0 = a0;
    o.arg1 = a1;
    o.arg2 = a2;
    o.arg3 = a3;
    o.arg4 = a4;
    o.name = static_cast<uint32_t>(ops.size());  // name ids follow the ops (one path per op)
    ops.push_back(o);
    return static_cast<uint32_t>(ops.size() - 1);
  }
  uint32_t add_table(const std::vector<uint32_t> &v) {
    const uint32_t i = static_cast<uint32_t>(table.size());
    table.insert(table.end(), v.begin(), v.end());
    return i;
  }
  void add_sub(type_t *t, uint32_t vec_op) {
    for (auto &s : subs)
      if (s.t == t) {
        s.vecs.push_back(vec_op);
        return;
      }
    subs.push_back({t, 0, {vec_op}});
    pending.push_back(subs.size() - 1);
  }

  static uint32_t stride(const type_t *t) { return align_up(t->size, t->align); }

  void walk(type_t *t, uint32_t noff, uint32_t depth) {
    switch (t->k) {
    case kind::scalar: emit(t->op, noff, depth); return;
    case kind::enm:
      if (t->validate)
        emit(XDRG_OP_ENUM, noff, depth, XDRG_F_VALIDATE, add_table(t->enum_vals),
             static_cast<uint32_t>(t->enum_vals.size()));
      else
        emit(XDRG_OP_ENUM, noff, depth);
      return;
    case kind::opaque_array: emit(XDRG_OP_OPAQUE, noff, depth, 0, t->n); return;
    case kind::varbytes: emit(t->op, noff, depth, 0, t->n); return;
    case kind::vd: return;
    case kind::unsupported: throw gen_error(t->name + ": " + t->why);
    case kind::xarray: {  // xarray<T,N>: a container level, N elements (types.h:424-452)
      const uint32_t step = stride(t->elem);
      for (uint32_t i = 0; i < t->n; ++i) walk(t->elem, noff + i * step, depth + 1);
      return;
    }
    case kind::xvector: {  // xvector<T,N> / pointer<T> (types.h:365-414, :591-665)
      const uint32_t d = depth + 1;
      const uint8_t flags = t->pointer ? XDRG_F_POINTER : 0;
      if (!t->elem->fixed) {
        const uint32_t v = emit(XDRG_OP_VECTOR, noff, d, flags | XDRG_F_SUB, t->n, stride(t->elem));
        add_sub(t->elem, v);
        return;
      }
      const uint32_t v = emit(XDRG_OP_VECTOR, noff, d, flags, t->n, stride(t->elem));
      const size_t start = ops.size();
      walk(t->elem, 0, d);  // element-relative offsets
      ops[v].arg2 = static_cast<uint32_t>(ops.size() - start);
      return;
    }
    case kind::strct:  // one class level (marshal.h:129-136), fields in order
      for (auto &f : t->fields) walk(f.t, noff + f.off, depth + 1);
      return;
    case kind::unn: {
      const uint32_t d = depth + 1;
      uint8_t flags = 0;
      uint32_t a0 = 0, a1 = 0;
      if (t->tag->k == kind::enm && t->tag->validate) {
        flags = XDRG_F_VALIDATE;
        a0 = add_table(t->tag->enum_vals);
        a1 = static_cast<uint32_t>(t->tag->enum_vals.size());
      }
      const uint32_t u = emit(XDRG_OP_UNION, noff, d, flags, a0, a1);
      msgs[u] = "bad value of " + t->tag_name + " in " + t->name;  // gen_hh.cc:479-481
      std::vector<std::pair<uint32_t, int64_t>> targets;  // (case, pc; -1 void)
      std::vector<uint32_t> jumps;
      const uint32_t base = noff + t->arms_off;
      for (auto &a : t->arms) {
        if (a.t->k == kind::vd) {
          for (uint32_t c : a.cases) targets.push_back({c, -1});
          continue;
        }
        const uint32_t pc = static_cast<uint32_t>(ops.size());
        walk(a.t, base, d);
        jumps.push_back(emit(XDRG_OP_JUMP, 0, d));
        for (uint32_t c : a.cases) targets.push_back({c, pc});
      }
      int64_t def_pc = -2;  // none
      if (t->has_default) {
        if (t->def.t->k == kind::vd) {
          def_pc = -1;
        } else {
          def_pc = static_cast<int64_t>(ops.size());
          walk(t->def.t, base, d);
          jumps.push_back(emit(XDRG_OP_JUMP, 0, d));
        }
      }
      const uint32_t end = static_cast<uint32_t>(ops.size());
      for (uint32_t j : jumps) ops[j].arg0 = end;
      std::vector<uint32_t> tab;
      for (auto &c : targets) {
        tab.push_back(c.first);
        tab.push_back(c.second < 0 ? end : static_cast<uint32_t>(c.second));
      }
      ops[u].arg2 = add_table(tab);
      ops[u].arg3 = static_cast<uint32_t>(targets.size());
      if (def_pc != -2) {
        ops[u].flags |= XDRG_F_DEFAULT;
        ops[u].arg4 = def_pc == -1 ? end : static_cast<uint32_t>(def_pc);
      }
      return;
    }
    }
  }

  void compile(type_t *root) {
    subs.push_back({root, 0, {}});  // the record's own ops serve as its subroutine (pc 0)
    walk(root, 0, 0);
    emit(XDRG_OP_END, 0, 0);
    while (!pending.empty()) {
      const size_t i = pending.front();  // (walk may append to subs)
      pending.pop_front();
      subs[i].entry = static_cast<uint32_t>(ops.size());
      walk(subs[i].t, 0, 0);  // element-relative offsets and depths
      emit(XDRG_OP_END, 0, 0);
    }
    for (auto &s : subs)
      for (uint32_t v : s.vecs) ops[v].arg4 = s.entry;
  }
};

// ------------------------------------------------------------ the symlist
class resolver {
 public:
  explicit resolver(const plan_gen_options &o) : opt_(o) {
    consts_["TRUE"] = 1;
    consts_["FALSE"] = 0;
    auto base = [&](const char *n, uint8_t op, uint32_t size, uint32_t wire) {
      type_t *t = make(kind::scalar);
      t->name = n;
      t->op = op;
      t->size = t->align = size;
      t->fixed = true;
      t->wire = wire;
      base_[n] = t;
    };
    base("int", XDRG_OP_U32, 4, 4);
    base("unsigned", XDRG_OP_U32, 4, 4);
    base("float", XDRG_OP_U32, 4, 4);
    base("hyper", XDRG_OP_U64, 8, 8);
    base("unsigned hyper", XDRG_OP_U64, 8, 8);
    base("double", XDRG_OP_U64, 8, 8);
    base("bool", XDRG_OP_BOOL, 1, 4);
    void_ = make(kind::vd);
    void_->fixed = true;
  }

  // Constants and enums in file order first; then every struct, union and
  // typedef (so a type may use a constant defined after it, as xdrc's C++
  // output allows).
  void load(const symlist_t &syms) {
    std::vector<std::string> ns;
    for (const rpc_sym &s : syms) {
      switch (s.gettype()) {
      case rpc_sym::NAMESPACE: ns.push_back(*s.sliteral); break;
      case rpc_sym::CLOSEBRACE: if (!ns.empty()) ns.pop_back(); break;
      case rpc_sym::CONST: consts_[s.sconst->id] = value(s.sconst->val); break;
      case rpc_sym::ENUM: {
        type_t *e = enum_type(*s.senum, qualify(ns, s.senum->id));
        types_[s.senum->id] = e;
        break;
      }
      case rpc_sym::STRUCT: decl_sym(s.sstruct->id, &s, qualify(ns, s.sstruct->id)); break;
      case rpc_sym::UNION: decl_sym(s.sunion->id, &s, qualify(ns, s.sunion->id)); break;
      case rpc_sym::TYPEDEF: decl_sym(s.stypedef->id, &s, qualify(ns, s.stypedef->id)); break;
      default: break;
      }
    }
    for (auto &n : order_) resolve(n);
  }

  // Every struct and union by name, typedefs naming one included, in file
  // order, with the qualified name of the declaration.
  struct record {
    std::string name, qualified;
    type_t *t;
  };
  std::vector<record> records() {
    std::vector<record> out;
    for (auto &n : order_) {
      type_t *t = types_.at(n);
      if (t->k == kind::strct || t->k == kind::unn) out.push_back({n, ast_.at(n).cxx, t});
    }
    return out;
  }
  bool is_typedef(const std::string &n) const { return typedefs_.count(n) != 0; }

 private:
  struct pending_sym {
    const rpc_sym *s;
    std::string cxx;
  };

  type_t *make(kind k) {
    pool_.push_back(std::make_unique<type_t>());
    pool_.back()->k = k;
    return pool_.back().get();
  }
  static std::string qualify(const std::vector<std::string> &ns, const std::string &id) {
    std::string q;
    for (auto &n : ns) q += "::" + n;
    return q + "::" + id;
  }
  void decl_sym(const std::string &id, const rpc_sym *s, const std::string &cxx) {
    ast_[id] = {s, cxx};
    order_.push_back(id);
    if (s->gettype() == rpc_sym::TYPEDEF) typedefs_.insert(id);
  }

  // A number (decimal, 0x hex, signed) or a constant / enum tag; signed, as
  // xdrc's C++ output reads it (case values and tables take it mod 2^32).
  int64_t value(const std::string &v) {
    if (!v.empty() && (std::isdigit(static_cast<unsigned char>(v[0])) || v[0] == '-' || v[0] == '+')) {
      char *end = nullptr;
      const long long x = std::strtoll(v.c_str(), &end, 0);
      if (end && *end == '\0') return x;
    }
    auto it = consts_.find(local_name(v));
    if (it == consts_.end()) throw gen_error("unknown constant '" + v + "'");
    return it->second;
  }

  type_t *enum_type(const rpc_enum &e, const std::string &cxx) {
    type_t *t = make(kind::enm);
    t->name = e.id;
    t->size = t->align = 4;
    t->fixed = true;
    t->wire = 4;
    int64_t next = 0;
    std::set<int64_t> vals;  // the table lists the tags in signed order
    for (const rpc_const &c : e.tags) {
      const int64_t v = c.val.empty() ? next : value(c.val);
      consts_[c.id] = v;
      vals.insert(v);
      next = v + 1;
    }
    for (int64_t v : vals) t->enum_vals.push_back(static_cast<uint32_t>(v));
    t->validate = opt_.validate_enums.count(e.id) != 0;
    if (!cxx.empty()) t->enums_cxx.push_back(cxx);
    return t;
  }

  type_t *resolve(const std::string &name) {
    auto it = types_.find(name);
    if (it != types_.end()) return it->second;
    auto a = ast_.find(name);
    if (a == ast_.end()) throw gen_error("unknown type '" + name + "'");
    const rpc_sym *s = a->second.s;
    if (busy_.count(name)) {  // a self-referential union or typedef (a struct may be: declared first)
      type_t *t = make(kind::unsupported);
      t->name = name;
      t->why = "recursive union or typedef: only structs may refer to themselves";
      t->size = 16;
      t->align = 8;
      return t;
    }
    if (s->gettype() == rpc_sym::STRUCT) {
      type_t *t = make(kind::strct);
      t->name = s->sstruct->id;
      t->cxx = a->second.cxx;
      types_[name] = t;
      define_struct(t, s->sstruct->decls);
      return t;
    }
    busy_.insert(name);
    type_t *t = nullptr;
    try {
      if (s->gettype() == rpc_sym::UNION) {
        t = union_type(*s->sunion);
        t->cxx = a->second.cxx;
      } else {
        t = decl_type(*s->stypedef);
      }
    } catch (...) {
      busy_.erase(name);
      throw;
    }
    busy_.erase(name);
    types_[name] = t;
    return t;
  }

  type_t *named(const std::string &n0) {
    std::string n = n0;
    if (n.compare(0, 7, "struct ") == 0) n = n.substr(7);  // typedef struct foo bar;
    const std::string ln = local_name(n);
    auto b = base_.find(ln);
    if (b != base_.end()) return b->second;
    if (n == "quadruple") throw gen_error("quadruple is not supported (no xdr_traits in xdrpp)");
    auto it = types_.find(ln);
    if (it != types_.end()) return it->second;
    if (ast_.count(ln)) return resolve(ln);
    throw gen_error("unknown type '" + n0 + "'");
  }

  // A field's type specifier: a name, or an inline enum/struct/union named
  // _<field>_t (rpc_decl::set_id, xdrc/xdrc.cc:44-61, has named it already).
  type_t *spec(const rpc_decl &d) {
    switch (d.ts_which) {
    case rpc_decl::TS_ENUM: return enum_type(*d.ts_enum, "");
    case rpc_decl::TS_STRUCT: {
      type_t *t = make(kind::strct);
      t->name = d.ts_struct->id;
      define_struct(t, d.ts_struct->decls);
      return t;
    }
    case rpc_decl::TS_UNION: return union_type(*d.ts_union);
    case rpc_decl::TS_ID: break;
    }
    return named(d.type);
  }

  type_t *decl_type(const rpc_decl &d) {
    if (d.type == "opaque" && d.ts_which == rpc_decl::TS_ID) {
      if (d.qual == rpc_decl::ARRAY) {
        type_t *t = make(kind::opaque_array);
        t->n = static_cast<uint32_t>(value(d.bound));
        t->size = t->n;
        t->align = 1;
        t->fixed = true;
        t->wire = (static_cast<uint64_t>(t->n) + 3) & ~3ull;
        return t;
      }
      return varbytes(XDRG_OP_VAROPAQUE, d.bound);
    }
    if (d.type == "string" && d.ts_which == rpc_decl::TS_ID) return varbytes(XDRG_OP_STRING, d.bound);
    if (d.type == "void" && d.ts_which == rpc_decl::TS_ID) return void_;
    type_t *e = spec(d);
    switch (d.qual) {
    case rpc_decl::ARRAY: {
      type_t *t = make(kind::xarray);
      t->elem = e;
      t->n = static_cast<uint32_t>(value(d.bound));
      t->align = e->align;
      t->size = align_up(e->size, e->align) * t->n;
      t->fixed = e->fixed;
      t->wire = e->wire * t->n;
      return t;
    }
    case rpc_decl::VEC: return vector(e, bound(d.bound), false);
    case rpc_decl::PTR: return vector(e, 1, true);
    case rpc_decl::SCALAR: break;
    }
    return e;
  }

  uint32_t bound(const std::string &b) { return b.empty() ? kMaxLen : static_cast<uint32_t>(value(b)); }
  type_t *varbytes(uint8_t op, const std::string &b) {
    type_t *t = make(kind::varbytes);
    t->op = op;
    t->n = bound(b);
    t->size = 16;  // xdrg_bytes_ref
    t->align = 8;
    return t;
  }
  type_t *vector(type_t *e, uint32_t max, bool ptr) {
    type_t *t = make(kind::xvector);
    t->elem = e;
    t->n = max;
    t->pointer = ptr;
    t->size = 16;  // xdrg_bytes_ref of the staged element array
    t->align = 8;
    return t;
  }

  // Natural alignment of the staged record (the C++ layout xdrc emits for
  // fixed-size types).
  void define_struct(type_t *t, const vec<rpc_decl> &decls) {
    uint32_t off = 0, al = 1;
    bool fixed = true;
    uint64_t wire = 0;
    for (const rpc_decl &d : decls) {
      type_t *ft = decl_type(d);
      off = align_up(off, ft->align);
      t->fields.push_back({d.id, ft, off});
      off += ft->size;
      al = std::max(al, ft->align);
      fixed = fixed && ft->fixed;
      wire += ft->wire;
    }
    t->align = al;
    t->size = t->fields.empty() ? 1 : align_up(std::max<uint32_t>(off, 1), al);
    t->fixed = fixed;
    t->wire = fixed ? wire : 0;
  }

  // Staged layout: {int32 tag; union of the arms} (include/xdrgpu.h).
  type_t *union_type(const rpc_union &u) {
    type_t *t = make(kind::unn);
    t->name = u.id;
    t->tag_name = u.tagid;
    t->tag = named(u.tagtype);
    uint32_t al = 4, sz = 0;
    for (const rpc_ufield &f : u.fields) {
      const bool is_void = f.decl.type == "void" && f.decl.ts_which == rpc_decl::TS_ID;
      type_t *at = is_void ? void_ : decl_type(f.decl);
      const std::string fname = is_void ? "" : f.decl.id;
      std::vector<uint32_t> vals;
      bool dflt = false;
      for (const std::string &c : f.cases) {
        if (c.empty()) dflt = true;  // `default:` (xdrc keeps it as an empty case)
        else vals.push_back(static_cast<uint32_t>(value(c)));
      }
      if (!vals.empty()) t->arms.push_back({vals, fname, at});
      if (dflt || f.hasdefault) {
        t->has_default = true;
        t->def = {{}, fname, at};
      }
      al = std::max(al, at->align);
      sz = std::max(sz, at->size);
    }
    t->arms_off = align_up(4, al);
    t->align = al;
    t->size = align_up(t->arms_off + sz, al);
    t->fixed = false;
    return t;
  }

  const plan_gen_options &opt_;
  std::vector<std::unique_ptr<type_t>> pool_;
  std::map<std::string, type_t *> base_, types_;
  std::map<std::string, int64_t> consts_;
  std::map<std::string, pending_sym> ast_;
  std::set<std::string> busy_, typedefs_;
  std::vector<std::string> order_;
  type_t *void_ = nullptr;
};

// The C++ enum types a plan validates or leaves unvalidated: the emitted
// header checks each against xdrpp's xdr_validate_enum opt-in.
void collect_enums(type_t *t, std::set<type_t *> &seen, std::vector<type_t *> &out) {
  if (!t || !seen.insert(t).second) return;
  if (t->k == kind::enm && !t->enums_cxx.empty()) out.push_back(t);
  collect_enums(t->elem, seen, out);
  collect_enums(t->tag, seen, out);
  for (auto &f : t->fields) collect_enums(f.t, seen, out);
  for (auto &a : t->arms) collect_enums(a.t, seen, out);
  if (t->has_default) collect_enums(t->def.t, seen, out);
}

// Top-level structs and unions a plan walks (their validate() hooks).
void collect_classes(type_t *t, std::set<type_t *> &seen, std::vector<type_t *> &out) {
  if (!t || !seen.insert(t).second) return;
  if ((t->k == kind::strct || t->k == kind::unn) && !t->cxx.empty()) out.push_back(t);
  collect_classes(t->elem, seen, out);
  for (auto &f : t->fields) collect_classes(f.t, seen, out);
  for (auto &a : t->arms) collect_classes(a.t, seen, out);
  if (t->has_default) collect_classes(t->def.t, seen, out);
}

// XDRG_PLAN_TYPES_<FILE>: the emitted types of file.x as an X-macro list.
std::string guard_macro(const std::string &input) {
  std::string b = input;
  const size_t k = b.rfind('/');
  if (k != std::string::npos) b = b.substr(k + 1);
  if (b.size() > 2 && b.compare(b.size() - 2, 2, ".x") == 0) b.resize(b.size() - 2);
  std::string m = "XDRG_PLAN_TYPES_";
  for (unsigned char ch : b) m += std::isalnum(ch) ? static_cast<char>(std::toupper(ch)) : '_';
  return m;
}

std::string cstr(const std::string &s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}

}  // namespace

int gen_plan(std::ostream &os, const symlist_t &syms, const plan_gen_options &opt) {
  resolver R(opt);
  R.load(syms);
  const std::string guard = opt.guard.empty() ? "XDRG_EMITTED_PLANS_H" : opt.guard;
  os << "/* Generated by xdrc -plan (xdrpp_amd/gen/gen_plan.cc)"
     << (opt.input.empty() ? "" : " from " + opt.input) << " -- do not edit.\n"
     << " * Device plans (include/xdrgpu.h xdrg_plan_create) of its structs and unions. */\n"
     << "#ifndef " << guard << "\n#define " << guard << " 1\n#include \"xdrgpu.h\"\n\n";
  std::ostringstream cxx;  // C++ emitted_plan<T> specializations
  int rc = 0;
  std::set<std::string> kernel_set(opt.kernel_types.begin(), opt.kernel_types.end());
  std::ostringstream types;  // X(C++ type, C identifier) of every emitted_plan
  for (auto &rec : R.records()) {
    const std::string &n = rec.name;
    type_t *t = rec.t;
    plan_ctx P;
    try {
      P.compile(t);
    } catch (const gen_error &e) {
      os << "/* " << n << ": no device plan (" << e.what() << ") */\n\n";
      continue;
    }
    // C names from the qualified declaration (testns::numerics ->
    // xdrg_plan_testns_numerics_ops): two files may declare one name in
    // different namespaces
    std::string q = rec.qualified.compare(0, 2, "::") == 0 ? rec.qualified.substr(2) : rec.qualified;
    for (size_t k; (k = q.find("::")) != std::string::npos;) q.replace(k, 2, "_");
    const std::string c = c_ident(q);
    std::string C = c;
    for (auto &ch : C) ch = static_cast<char>(std::toupper(static_cast<unsigned char>(ch)));
    const uint32_t stride = align_up(std::max<uint32_t>(t->size, 1), t->align);
    os << "/* " << n << ": " << P.ops.size() << " ops, stride " << stride << ", "
       << (t->fixed ? "fixed " + std::to_string(t->wire) + " wire bytes" : std::string("variable length"))
       << " */\n";
    os << "static const xdrg_op xdrg_plan_" << c << "_ops[" << P.ops.size() << "] = {\n";
    for (const xdrg_op &o : P.ops)
      os << "  {" << unsigned(o.kind) << ", " << unsigned(o.flags) << ", " << o.depth << ", " << o.noff << "u, "
         << o.arg0 << "u, " << o.arg1 << "u, " << o.arg2 << "u, " << o.arg3 << "u, " << o.arg4 << "u, " << o.name
         << "u},\n";
    os << "};\n";
    std::vector<uint32_t> tab = P.table;
    if (tab.empty()) tab.push_back(0);
    os << "static const uint32_t xdrg_plan_" << c << "_table[" << tab.size() << "] = {\n";
    for (size_t i = 0; i < tab.size(); i += 8) {
      os << " ";
      for (size_t j = i; j < std::min(tab.size(), i + 8); ++j) os << " " << tab[j] << "u,";
      os << "\n";
    }
    os << "};\n";
    os << "#define XDRG_PLAN_" << C << "_NOPS " << P.ops.size() << "u\n"
       << "#define XDRG_PLAN_" << C << "_NTABLE " << P.table.size() << "u\n"
       << "#define XDRG_PLAN_" << C << "_STRIDE " << stride << "u\n"
       << "#define XDRG_PLAN_" << C << "_FIXED_SIZE " << (t->fixed ? t->wire : 0) << "u\n";
    if (!P.msgs.empty()) {
      os << "static const struct { uint32_t op; const char *what; } xdrg_plan_" << c << "_union_msgs["
         << P.msgs.size() << "] = {\n";
      for (auto &m : P.msgs) os << "  {" << m.first << "u, " << cstr(m.second) << "},\n";
      os << "};\n";
    }
    os << "static inline int xdrg_plan_create_" << c << "(xdrg_plan **out) {\n"
       << "  return xdrg_plan_create(xdrg_plan_" << c << "_ops, XDRG_PLAN_" << C << "_NOPS, xdrg_plan_" << c
       << "_table, XDRG_PLAN_" << C << "_NTABLE, XDRG_PLAN_" << C << "_STRIDE, out);\n}\n";
    // the plan-specialized kernels, written now for hipcc at build time
    std::string kstem;
    if (!opt.kernel_dir.empty() && !t->fixed && (kernel_set.empty() || kernel_set.count(n))) {
      xdrg_plan *h = nullptr;
      size_t len = 0;
      int e = xdrg_plan_create(P.ops.data(), static_cast<uint32_t>(P.ops.size()),
                               P.table.empty() ? nullptr : P.table.data(), static_cast<uint32_t>(P.table.size()),
                               stride, &h);
      if (!e) e = xdrg_plan_kernel_source(h, nullptr, 0, &len);
      std::string src(len + 1, '\0');
      if (!e) e = xdrg_plan_kernel_source(h, &src[0], src.size(), &len);
      if (h) xdrg_plan_destroy(h);
      if (e) {
        os << "/* " << n << ": no kernel source (" << e << ") */\n";
        rc = 1;
      } else {
        src.resize(len);
        std::ofstream f(opt.kernel_dir + "/" + c + ".hip");
        f << src;
        kstem = c;
      }
    }
    if (!kstem.empty()) os << "#define XDRG_PLAN_" << C << "_KERNELS " << cstr(kstem) << "\n";
    os << "\n";
    // C++: the plan plan_for<T>() takes (only for the type's own name: a
    // typedef names the same C++ type)
    if (t->cxx.empty() || R.is_typedef(n)) continue;
    std::set<type_t *> seen;
    std::vector<type_t *> enums, classes;
    collect_enums(t, seen, enums);
    seen.clear();
    collect_classes(t, seen, classes);
    types << " \\\n  X(" << t->cxx << ", " << c << ")";
    cxx << "template <> struct emitted_plan<" << t->cxx << "> {\n"
        << "  static constexpr const xdrg_op *ops = xdrg_plan_" << c << "_ops;\n"
        << "  static constexpr std::uint32_t nops = XDRG_PLAN_" << C << "_NOPS;\n"
        << "  static constexpr const std::uint32_t *table = xdrg_plan_" << c << "_table;\n"
        << "  static constexpr std::uint32_t ntable = XDRG_PLAN_" << C << "_NTABLE;\n"
        << "  static constexpr std::uint32_t stride = XDRG_PLAN_" << C << "_STRIDE;\n"
        << "  static constexpr bool fixed = " << (t->fixed ? "true" : "false") << ";\n"
        << "  static constexpr const char *kernels = " << cstr(kstem) << ";\n"
        << "  static constexpr bool validates = false";
    for (type_t *k : classes) cxx << "\n      || xdrg_validate_probe::has_hook<" << k->cxx << ">";
    cxx << ";\n  static std::vector<std::pair<std::uint32_t, std::string>> msgs() {\n    return {";
    bool first = true;
    for (auto &m : P.msgs) {
      cxx << (first ? "" : ", ") << "{" << m.first << "u, " << cstr(m.second) << "}";
      first = false;
    }
    cxx << "};\n  }\n};\n";
    for (type_t *e : enums)
      cxx << "static_assert(detail::enum_validates<" << e->enums_cxx[0] << ">::value == "
          << (e->validate ? "true" : "false") << ", \"" << e->enums_cxx[0]
          << ": xdr_validate_enum opt-in differs from the emitted plan (xdrc -plan -validate)\");\n";
  }
  const std::string xguard = opt.xdr_guard;
  if (!cxx.str().empty() && !xguard.empty())
    os << "#if defined(__cplusplus) && defined(XDRPP_GPU_HH_INCLUDED) && defined(" << xguard << ")\n"
       << "/* xdr::gpu::plan_for<T>() takes these instead of recording the plan from\n"
       << " * xdr_traits<T> (include/xdrpp_gpu.hh): the types xdrc -hh emitted for the\n"
       << " * same file are visible here. */\n"
       << "namespace xdr {\nnamespace gpu {\n"
       << cxx.str() << "}  // namespace gpu\n}  // namespace xdr\n"
       << "/* X(C++ type, C name) for every type above */\n"
       << "#define " << guard_macro(opt.input) << "(X)" << types.str() << "\n#endif\n";
  os << "#endif /* " << guard << " */\n";
  return rc;
}

}  // namespace xdrg_gen
