// -*- C++ -*-
// xdrpp_gpu.hh — header-only C++ layer of the MI355X batched XDR engine.
//
// Host code that uses xdrpp's xdrc-generated xdr_traits<T> keeps doing so;
// this header turns xdr_traits<T> into a device plan and calls libxdrgpu.so
// through the C ABI (xdrgpu.h).  Requires the xdrpp headers (<xdrpp/types.h>,
// <xdrpp/marshal.h>) and the HIP runtime headers.
//
//   xdr::gpu::to_opaque_batch(recs, n)        == xdr::xdr_to_opaque(r0, ..., rn-1)
//                                                (xdrpp/marshal.h:264-272)
//   xdr::gpu::from_opaque_batch(bytes, out, n) == xdr::xdr_from_opaque(bytes, r0, ..., rn-1)
//                                                (xdrpp/marshal.h:299-306)
//
// with the reference's exception classes and what() strings
// (xdrpp/types.h:57-99) and its marshaling_stack_limit (marshal.h:21,34).
//
// How the plan is obtained (plan_for<T>()): a recorder Archive walks
// xdr_traits<T>::save on a prototype object, field by field, exactly as
// xdr_generic_put does (marshal.h:110-136).  Unions are recorded arm by arm
// by driving xdr_traits<U>::load with each candidate discriminant
// (xdrc/gen_hh.cc:661-673): the candidates come from the discriminant's
// enum_values() (gen_hh.cc:271-305), or from U::_xdr_case_values()
// (gen_hh.cc:410-432), or from a union_cases<U> specialization.  The
// "bad value of <tag> in <union>" string is taken from the reference's own
// exception by loading one invalid discriminant.
//
// Staged layout.  A device record holds every field at natural alignment;
// opaque<>/string<> fields become xdrg_bytes_ref into a byte heap.  For
// fixed-size, trivially copyable types whose C++ layout already IS that
// layout (e.g. structs of ints/hypers/doubles) records are passed as-is;
// other types are staged/unstaged on the host by plan-following archives.
//
// Containers of variable-size elements (xvector<T>/pointer<T> of strings,
// structs with bytes fields, unions, containers -- and recursive types such
// as tests/xdrtest.x's test_recursive) give the element a subroutine
// (XDRG_F_SUB): its ops are recorded once per element type and placed after
// the record's END; a type still being recorded is referenced by key and
// patched when the plan is assembled.
#ifndef XDRPP_GPU_HH_INCLUDED
#define XDRPP_GPU_HH_INCLUDED 1

#include <xdrpp/marshal.h>
#include <xdrpp/types.h>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <typeindex>
#include <utility>
#include <vector>

#include "xdrgpu.h"

// Does a user validate() hook exist for T?  xdrc's load() ends every struct
// and union with `using xdr::validate; validate(obj);` (xdrc/gen_hh.cc:
// 244-247, :671-672): an overload found by argument-dependent lookup, or a
// T::validate() member that xdr::validate calls (xdrpp/types.h:109-140).
// Ordinary lookup here finds only the probe's own template, so the call
// resolves to a user overload when there is one (a non-template exact
// match) and to the probe (or ambiguously, for types in namespace xdr, to
// xdr::validate) when there is none.
namespace xdrg_validate_probe {
struct no_hook {};
template <typename T> no_hook validate(const T &);
template <typename T, typename = void> struct adl : std::false_type {};
template <typename T>
struct adl<T, std::void_t<decltype(validate(std::declval<const T &>()))>>
    : std::bool_constant<!std::is_same_v<decltype(validate(std::declval<const T &>())), no_hook>> {};
template <typename T, typename = void> struct member : std::false_type {};
template <typename T>
struct member<T, std::void_t<decltype(std::declval<const T &>().validate())>> : std::true_type {};
template <typename T> constexpr bool has_hook = adl<T>::value || member<T>::value;
}  // namespace xdrg_validate_probe

namespace xdr {
namespace gpu {

//! Customization point: the case values of union U and whether it has a
//! default arm.  The primary template uses what xdrc generates.
template <typename U, typename = void> struct union_cases {
  static std::vector<std::int64_t> values();
  static constexpr bool has_default = U::_xdr_has_default_case;
};

//! Plans emitted at generation time: `xdrc -plan file.x` (the plan back end,
//! xdrpp_amd/gen/gen_plan.cc) writes file_plan.hh, which specializes this
//! for every struct and union of file.x when it is included after this
//! header and after file.hh (xdrc -hh).  plan_for<T>() then takes the
//! emitted tables -- nothing is recorded from xdr_traits<T> at run time --
//! and, when the emitted plan names a code object (`-kernels`, compiled by
//! hipcc at build time) found in $XDRG_PLAN_KERNEL_DIR or
//! XDRG_EMITTED_KERNEL_DIR, attaches the plan-specialized kernels too.
template <typename T> struct emitted_plan;

//! API-level failure of the C ABI (bad arguments, HIP error).
struct api_error : std::runtime_error {
  int code;
  api_error(int c, const std::string &what) : std::runtime_error(what), code(c) {}
};

namespace detail {

inline std::uint32_t align_up(std::uint32_t x, std::uint32_t a) { return (x + a - 1) / a * a; }

// Buffers the batch calls allocate (pinned host and device), counted so
// that a test can see a context reach its steady state (no allocation).
inline std::atomic<std::size_t> &alloc_count() {
  static std::atomic<std::size_t> c{0};
  return c;
}

//! Pinned (page-locked) host memory for std::vector: the staged records and
//! heaps are copied to and from the device by DMA, asynchronously.
template <typename T> struct pinned_allocator {
  using value_type = T;
  pinned_allocator() = default;
  template <typename U> pinned_allocator(const pinned_allocator<U> &) {}
  T *allocate(std::size_t n) {
    void *p = nullptr;
    const hipError_t e = hipHostMalloc(&p, std::max<std::size_t>(n, 1) * sizeof(T), hipHostMallocDefault);
    if (e != hipSuccess) throw api_error(XDRG_EHIP, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    ++alloc_count();
    return static_cast<T *>(p);
  }
  void deallocate(T *p, std::size_t) { (void)hipHostFree(p); }
  template <typename U> bool operator==(const pinned_allocator<U> &) const { return true; }
  template <typename U> bool operator!=(const pinned_allocator<U> &) const { return false; }
};
using host_bytes = std::vector<std::uint8_t, pinned_allocator<std::uint8_t>>;

// ---------------------------------------------------------------- type tests
template <typename T> struct bytes_kind {
  static constexpr int kind = 0;
  static constexpr std::uint32_t n = 0;
};
template <std::uint32_t N> struct bytes_kind<opaque_array<N>> {
  static constexpr int kind = XDRG_OP_OPAQUE;
  static constexpr std::uint32_t n = N;
};
template <std::uint32_t N> struct bytes_kind<xvector<std::uint8_t, N>> {
  static constexpr int kind = XDRG_OP_VAROPAQUE;
  static constexpr std::uint32_t n = N;
};
template <std::uint32_t N> struct bytes_kind<xstring<N>> {
  static constexpr int kind = XDRG_OP_STRING;
  static constexpr std::uint32_t n = N;
};
// xvector<T,N> (T not a byte) and pointer<T>: counted / optional containers
template <typename T> struct vector_info : std::false_type {};
template <typename E, std::uint32_t N> struct vector_info<xvector<E, N>> : std::true_type {
  using elem = E;
  static constexpr std::uint32_t max = N;
  static constexpr bool pointer = false;
};
template <std::uint32_t N> struct vector_info<xvector<std::uint8_t, N>> : std::false_type {};
template <typename E> struct vector_info<pointer<E>> : std::true_type {
  using elem = E;
  static constexpr std::uint32_t max = 1;
  static constexpr bool pointer = true;
};
template <typename T> struct xarray_info : std::false_type {};
template <typename E, std::uint32_t N> struct xarray_info<xarray<E, N>> : std::true_type {
  using elem = E;
  static constexpr std::uint32_t n = N;
};

// enum validation opt-in: the same test validate_enum<T> makes
// (xdrpp/types.h:157-173).
template <typename E> struct enum_validated {
  template <typename U> static std::false_type test(...);
  template <typename U> static decltype(xdr_validate_enum(U{}), std::true_type{}) test(int);
  static constexpr bool value = decltype(test<E>(0))::value;
};

template <typename E> using enum_validates = enum_validated<E>;  // (emitted plan headers)

// T has an emitted plan (a complete emitted_plan<T> specialization)
template <typename T, typename = void> struct has_emitted_plan : std::false_type {};
template <typename T>
struct has_emitted_plan<T, std::void_t<decltype(emitted_plan<T>::nops)>> : std::true_type {};

// Plans recorded from xdr_traits at run time (tests: an emitted plan records none)
inline std::atomic<std::size_t> &recorded_plans() {
  static std::atomic<std::size_t> c{0};
  return c;
}

template <typename U, typename = void> struct has_case_values : std::false_type {};
template <typename U>
struct has_case_values<U, std::void_t<decltype(U::_xdr_case_values())>> : std::true_type {};

template <typename T> using plain = std::remove_cv_t<std::remove_reference_t<T>>;

// The declared discriminant type of a union: xdr_traits<U>::discriminant_type
// (xdrc emits it, gen_hh.cc), else what _xdr_discriminant() returns.
template <typename U, typename = void> struct discriminant_of {
  using type = decltype(std::declval<U>()._xdr_discriminant());
};
template <typename U>
struct discriminant_of<U, std::void_t<typename xdr_traits<U>::discriminant_type>> {
  using type = typename xdr_traits<U>::discriminant_type;
};

// ---------------------------------------------------------------- sub-plans
// Ops of one type placed at offset 0, pcs relative to the sub-plan start,
// depths relative to the level the type is placed at.
struct subplan {
  std::vector<xdrg_op> ops;
  std::vector<std::uint32_t> table;
  std::vector<std::pair<std::uint32_t, std::string>> msgs;  // op -> bad-discriminant what()
  std::uint32_t size = 0, align = 1;
  bool identity = true;  // staged layout == C++ layout of the type
  bool fixed = true;     // fixed wire size (xdr_traits<T>::has_fixed_size)
  bool validates = false;  // some struct/union in the type has a validate() hook

  bool same_ops(const subplan &o) const {
    if (ops.size() != o.ops.size() || table != o.table) return false;
    for (std::size_t i = 0; i < ops.size(); ++i)
      if (std::memcmp(&ops[i], &o.ops[i], sizeof(xdrg_op)) != 0) return false;
    return true;
  }
};

inline xdrg_op mkop(int kind, std::uint32_t noff, std::uint16_t depth, std::uint32_t a0 = 0,
                    std::uint32_t a1 = 0, std::uint8_t flags = 0) {
  xdrg_op o{};
  o.kind = static_cast<std::uint8_t>(kind);
  o.flags = flags;
  o.depth = depth;
  o.noff = noff;
  o.arg0 = a0;
  o.arg1 = a1;
  return o;
}

// Append `src` to `dst` at byte offset `base`, `dadd` levels deeper.
inline void append(subplan &dst, const subplan &src, std::uint32_t base, std::uint16_t dadd) {
  const std::uint32_t pc0 = static_cast<std::uint32_t>(dst.ops.size());
  const std::uint32_t t0 = static_cast<std::uint32_t>(dst.table.size());
  dst.table.insert(dst.table.end(), src.table.begin(), src.table.end());
  std::uint32_t body = 0;  // ops left in a VECTOR body (element-relative offsets)
  for (xdrg_op o : src.ops) {
    if (body) --body;
    else if (o.kind != XDRG_OP_JUMP) o.noff += base;
    if (o.kind == XDRG_OP_VECTOR) body = o.arg2;
    o.depth = static_cast<std::uint16_t>(o.depth + dadd);
    if (o.kind == XDRG_OP_JUMP) o.arg0 += pc0;
    if ((o.kind == XDRG_OP_ENUM || o.kind == XDRG_OP_UNION) && (o.flags & XDRG_F_VALIDATE))
      o.arg0 += t0;
    if (o.kind == XDRG_OP_UNION) {
      o.arg2 += t0;
      for (std::uint32_t c = 0; c < o.arg3; ++c) dst.table[o.arg2 + 2 * c + 1] += pc0;
      if (o.flags & XDRG_F_DEFAULT) o.arg4 += pc0;
    }
    dst.ops.push_back(o);
  }
  for (const auto &m : src.msgs) dst.msgs.emplace_back(m.first + pc0, m.second);
}

template <typename T> subplan record_type();

// Element subroutines of the plan being assembled (batch_plan): one body
// per element type.  `busy` holds the struct/union types whose recording is
// on the stack: an element of such a type (a recursive type) is known to be
// variable-size and is referenced before its body exists.  F_SUB VECTOR ops
// carry the body's key in arg4 until the plan is assembled.
struct sub_registry {
  std::vector<std::type_index> types;
  std::vector<subplan> bodies;
  std::vector<std::type_index> busy;
};
inline sub_registry *&active_subs() {
  static thread_local sub_registry *r = nullptr;
  return r;
}
struct busy_guard {
  explicit busy_guard(std::type_index t) {
    if (active_subs()) active_subs()->busy.push_back(t);
  }
  ~busy_guard() {
    if (active_subs()) active_subs()->busy.pop_back();
  }
};
template <typename E> bool recording() {
  const sub_registry *R = active_subs();
  return R && std::find(R->busy.begin(), R->busy.end(), std::type_index(typeid(E))) != R->busy.end();
}
template <typename E> std::uint32_t sub_key() {
  sub_registry *R = active_subs();
  if (!R) throw std::logic_error("xdr::gpu: element subroutines are recorded by plan_for<T>()");
  const std::type_index t(typeid(E));
  for (std::size_t k = 0; k < R->types.size(); ++k)
    if (R->types[k] == t) return static_cast<std::uint32_t>(k);
  const std::uint32_t k = static_cast<std::uint32_t>(R->types.size());
  R->types.push_back(t);  // before recording: the body may refer to itself
  R->bodies.emplace_back();
  subplan b = record_type<E>();
  R->bodies[k] = std::move(b);
  return k;
}

// Walks xdr_traits<S>::save on a prototype: each archived field is placed
// at its natural alignment (the C++ rule xdrc structs follow).
struct struct_recorder {
  subplan *sp;
  const char *proto;
  std::uint32_t off = 0;
  template <typename F> void operator()(const F &f) {
    const subplan fp = record_type<plain<F>>();
    off = align_up(off, fp.align);
    const std::uintptr_t cxx = reinterpret_cast<const char *>(&f) - proto;
    if (cxx != off || !fp.identity) sp->identity = false;
    append(*sp, fp, off, 1);  // class level (marshal.h:129-136)
    off += fp.size;
    sp->align = std::max(sp->align, fp.align);
    sp->fixed = sp->fixed && fp.fixed;
    sp->validates = sp->validates || fp.validates;
  }
};

// Drives xdr_traits<U>::load: the first archived value is the discriminant
// (fed `disc`), the next (if any) is the selected arm.
struct union_feeder {
  std::int64_t disc;
  int seen = 0;
  bool disc_validated = false;
  std::vector<std::int32_t> disc_values;  // when validated
  subplan arm;
  bool have_arm = false;
  template <typename F> void operator()(F &f) {
    using P = plain<F>;
    if (seen++ == 0) {
      if constexpr (std::is_integral_v<P> || std::is_enum_v<P>) {
        f = static_cast<P>(disc);
        if constexpr (xdr_traits<P>::is_enum && !std::is_same_v<P, bool>) {
          if constexpr (enum_validated<P>::value) {
            disc_validated = true;
            for (std::int32_t v : xdr_traits<P>::enum_values()) disc_values.push_back(v);
          }
        }
      } else {
        throw std::logic_error("xdr::gpu: union discriminant is not a 32-bit integer");
      }
      return;
    }
    if (have_arm) throw std::logic_error("xdr::gpu: union load archived two arms");
    arm = record_type<P>();
    have_arm = true;
  }
};

}  // namespace detail

template <typename U, typename E>
std::vector<std::int64_t> union_cases<U, E>::values() {
  std::vector<std::int64_t> v;
  if constexpr (detail::has_case_values<U>::value)
    for (auto c : U::_xdr_case_values()) v.push_back(static_cast<std::int64_t>(c));
  return v;
}

namespace detail {

template <typename U> subplan record_union() {
  const busy_guard busy{std::type_index(typeid(U))};
  // candidate discriminants: union_cases<U>, else the discriminant enum's tags
  std::vector<std::int64_t> cand = union_cases<U>::values();
  const bool has_default = union_cases<U>::has_default;
  if constexpr (has_case_values<U>::value) {
    if (cand.empty()) {  // xdrc lists no cases for unions with a default arm:
      // the tags of the discriminant's enum (xdr_traits<U>::discriminant_type)
      using D = plain<typename discriminant_of<U>::type>;
      if constexpr (xdr_traits<D>::is_enum)
        for (auto v : xdr_traits<D>::enum_values()) cand.push_back(v);
    }
  }
  if (cand.empty())
    throw std::logic_error("xdr::gpu: cannot enumerate the cases of a union (specialize xdr::gpu::union_cases)");
  std::int64_t probe = 0;
  for (auto v : cand) probe = std::max(probe, v + 1);

  struct arm_rec { bool is_void; subplan sp; };
  std::vector<std::pair<std::int64_t, arm_rec>> cases;
  bool validated = false;
  std::vector<std::int32_t> vvals;
  std::string message;
  auto run = [&](std::int64_t v, arm_rec &out) -> bool {
    U u{};
    union_feeder f{v};
    try {
      xdr_traits<U>::load(f, u);
    } catch (const xdr_bad_discriminant &e) {
      message = e.what();
      return false;
    }
    validated = f.disc_validated;
    vvals = f.disc_values;
    out.is_void = !f.have_arm;
    if (f.have_arm) out.sp = std::move(f.arm);
    return true;
  };
  arm_rec dflt{};
  bool have_dflt = false;
  if (has_default) have_dflt = run(probe, dflt);
  for (auto v : cand) {
    arm_rec a{};
    if (!run(v, a)) continue;
    if (have_dflt && a.is_void == dflt.is_void && (a.is_void || a.sp.same_ops(dflt.sp))) continue;
    cases.emplace_back(v, std::move(a));
  }
  if (!has_default) {
    arm_rec junk{};
    run(probe, junk);  // the reference's own "bad value of <tag> in <union>"
  }

  subplan sp;
  sp.fixed = false;
  sp.identity = false;
  std::uint32_t aal = 4, asz = 0;
  sp.validates = xdrg_validate_probe::has_hook<U>;
  auto grow = [&](const arm_rec &a) {
    if (!a.is_void) {
      aal = std::max(aal, a.sp.align);
      asz = std::max(asz, a.sp.size);
      sp.validates = sp.validates || a.sp.validates;
    }
  };
  for (auto &c : cases) grow(c.second);
  if (have_dflt) grow(dflt);
  const std::uint32_t arms_off = align_up(4, aal);
  sp.align = aal;
  sp.size = align_up(arms_off + asz, aal);

  std::uint8_t flags = 0;
  std::uint32_t a0 = 0, a1 = 0;
  if (validated) {
    flags |= XDRG_F_VALIDATE;
    a0 = static_cast<std::uint32_t>(sp.table.size());
    std::vector<std::int32_t> s(vvals);
    std::sort(s.begin(), s.end());
    s.erase(std::unique(s.begin(), s.end()), s.end());
    for (auto v : s) sp.table.push_back(static_cast<std::uint32_t>(v));
    a1 = static_cast<std::uint32_t>(s.size());
  }
  sp.ops.push_back(mkop(XDRG_OP_UNION, 0, 1, a0, a1, flags));
  if (!message.empty() && !has_default) sp.msgs.emplace_back(0, message);

  // arms, each once; identical arms share code
  std::vector<std::pair<std::int64_t, std::int64_t>> targets;  // (value, pc or -1 = end)
  std::vector<std::uint32_t> jumps;
  std::vector<std::pair<const subplan *, std::uint32_t>> placed;
  auto place = [&](const arm_rec &a) -> std::int64_t {
    if (a.is_void) return -1;
    for (auto &p : placed)
      if (p.first->same_ops(a.sp)) return p.second;
    const std::uint32_t pc = static_cast<std::uint32_t>(sp.ops.size());
    append(sp, a.sp, arms_off, 1);
    jumps.push_back(static_cast<std::uint32_t>(sp.ops.size()));
    sp.ops.push_back(mkop(XDRG_OP_JUMP, 0, 1));
    placed.emplace_back(&a.sp, pc);
    return pc;
  };
  for (auto &c : cases) targets.emplace_back(c.first, place(c.second));
  std::int64_t dpc = 0;
  if (have_dflt) dpc = place(dflt);
  const std::uint32_t end = static_cast<std::uint32_t>(sp.ops.size());
  for (auto j : jumps) sp.ops[j].arg0 = end;
  xdrg_op &u = sp.ops[0];
  u.arg2 = static_cast<std::uint32_t>(sp.table.size());
  u.arg3 = static_cast<std::uint32_t>(targets.size());
  for (auto &t : targets) {
    sp.table.push_back(static_cast<std::uint32_t>(t.first));
    sp.table.push_back(t.second < 0 ? end : static_cast<std::uint32_t>(t.second));
  }
  if (have_dflt) {
    u.flags |= XDRG_F_DEFAULT;
    u.arg4 = dpc < 0 ? end : static_cast<std::uint32_t>(dpc);
  }
  return sp;
}

template <typename T> subplan record_type() {
  using TR = xdr_traits<T>;
  subplan sp;
  if constexpr (std::is_same_v<T, bool>) {
    sp.ops.push_back(mkop(XDRG_OP_BOOL, 0, 0));
    sp.size = sp.align = 1;
  } else if constexpr (bytes_kind<T>::kind != 0) {
    constexpr int k = bytes_kind<T>::kind;
    sp.ops.push_back(mkop(k, 0, 0, bytes_kind<T>::n));
    if constexpr (k == XDRG_OP_OPAQUE) {
      sp.size = bytes_kind<T>::n;
      sp.align = 1;
    } else {
      sp.size = sizeof(xdrg_bytes_ref);
      sp.align = alignof(xdrg_bytes_ref);
      sp.identity = false;
      sp.fixed = false;
    }
  } else if constexpr (TR::is_enum) {
    static_assert(sizeof(T) == 4, "XDR enums are 32-bit");
    if constexpr (enum_validated<T>::value) {
      std::vector<std::int32_t> s(TR::enum_values().begin(), TR::enum_values().end());
      std::sort(s.begin(), s.end());
      s.erase(std::unique(s.begin(), s.end()), s.end());
      for (auto v : s) sp.table.push_back(static_cast<std::uint32_t>(v));
      sp.ops.push_back(mkop(XDRG_OP_ENUM, 0, 0, 0, static_cast<std::uint32_t>(s.size()),
                            XDRG_F_VALIDATE));
    } else {
      sp.ops.push_back(mkop(XDRG_OP_ENUM, 0, 0));
    }
    sp.size = sp.align = 4;
  } else if constexpr (TR::is_numeric) {
    using UT = typename TR::uint_type;
    sp.ops.push_back(mkop(sizeof(UT) == 8 ? XDRG_OP_U64 : XDRG_OP_U32, 0, 0));
    sp.size = sizeof(T);
    sp.align = alignof(T);
  } else if constexpr (vector_info<T>::value) {
    using E = typename vector_info<T>::elem;
    const std::uint8_t fl = vector_info<T>::pointer ? XDRG_F_POINTER : 0;
    sp.size = sizeof(xdrg_bytes_ref);
    sp.align = alignof(xdrg_bytes_ref);
    sp.identity = false;
    sp.fixed = false;
    subplan e;
    const bool inline_elems = !recording<E>() && (e = record_type<E>()).fixed;
    if (inline_elems) {  // fixed-size elements: ops inline after the VECTOR op
      xdrg_op v = mkop(XDRG_OP_VECTOR, 0, 1, vector_info<T>::max, align_up(e.size, e.align), fl);
      v.arg2 = static_cast<std::uint32_t>(e.ops.size());
      sp.ops.push_back(v);
      append(sp, e, 0, 1);  // elements inside the container level
      sp.validates = e.validates;
    } else {  // the element's subroutine; stride and body pc set by batch_plan
      xdrg_op v = mkop(XDRG_OP_VECTOR, 0, 1, vector_info<T>::max, 0, fl | XDRG_F_SUB);
      v.arg4 = sub_key<E>();
      sp.ops.push_back(v);
    }
  } else if constexpr (xarray_info<T>::value) {
    using E = typename xarray_info<T>::elem;
    const subplan e = record_type<E>();
    const std::uint32_t step = align_up(e.size, e.align);
    for (std::uint32_t i = 0; i < xarray_info<T>::n; ++i) append(sp, e, i * step, 1);  // container level
    sp.size = step * xarray_info<T>::n;
    sp.align = e.align;
    sp.identity = e.identity && sizeof(E) == step && sizeof(T) == sp.size;
    sp.fixed = e.fixed;
    sp.validates = e.validates;
  } else if constexpr (TR::is_union) {
    sp = record_union<T>();
  } else if constexpr (TR::is_struct || TR::is_class) {
    const busy_guard busy{std::type_index(typeid(T))};
    static const T proto{};
    struct_recorder r{&sp, reinterpret_cast<const char *>(&proto)};
    TR::save(r, proto);
    sp.size = align_up(std::max<std::uint32_t>(r.off, 1), sp.align);
    sp.validates = sp.validates || xdrg_validate_probe::has_hook<T>;
    if (sizeof(T) != sp.size || !std::is_trivially_copyable_v<T>) sp.identity = false;
  } else {
    static_assert(!sizeof(T *), "xdr::gpu: xvector<T>/pointer<T> of non-bytes T is not supported yet");
  }
  return sp;
}

// ------------------------------------------------- plan-following archives
// Stage: xdr_traits<T>::save writes the staged record + heap.
// Unstage: xdr_traits<T>::load reads them back.  Both follow the plan's
// pc in step with the archive calls (wire order), so every field lands at
// the op's staged offset; union discriminants pick the arm's pc.
struct cursor {
  const xdrg_op *ops;
  const std::uint32_t *table;
  std::uint32_t pc = 0;
  const xdrg_op &next() {
    while (ops[pc].kind == XDRG_OP_JUMP) pc = ops[pc].arg0;
    return ops[pc];
  }
  void branch(const xdrg_op &u, std::int32_t d) {
    for (std::uint32_t c = 0; c < u.arg3; ++c)
      if (static_cast<std::int32_t>(table[u.arg2 + 2 * c]) == d) { pc = table[u.arg2 + 2 * c + 1]; return; }
    if (u.flags & XDRG_F_DEFAULT) { pc = u.arg4; return; }
    throw xdr_bad_discriminant("bad value of discriminant");  // save() threw already
  }
};

template <typename V> struct stager : cursor {  // V: the heap's byte vector type
  std::uint8_t *rec = nullptr;  // the record, or (in_heap) heap offset `roff`
  V *heap;
  bool in_heap = false;
  std::uint64_t roff = 0;
  // the object's bytes, looked up at every write: staging elements grows the heap
  std::uint8_t *R() const { return in_heap ? heap->data() + roff : rec; }
  template <typename F> void operator()(const F &f) {
    using P = plain<F>;
    using TR = xdr_traits<P>;
    if constexpr (std::is_same_v<P, bool>) {
      R()[next().noff] = f ? 1 : 0;
      ++pc;
    } else if constexpr (bytes_kind<P>::kind == XDRG_OP_OPAQUE) {
      std::memcpy(R() + next().noff, f.data(), f.size());
      ++pc;
    } else if constexpr (bytes_kind<P>::kind != 0) {
      xdrg_bytes_ref r{heap->size(), static_cast<std::uint32_t>(f.size()), 0};
      heap->insert(heap->end(), reinterpret_cast<const std::uint8_t *>(f.data()),
                   reinterpret_cast<const std::uint8_t *>(f.data()) + f.size());
      std::memcpy(R() + next().noff, &r, sizeof r);
      ++pc;
    } else if constexpr (TR::is_enum || TR::is_numeric) {
      const xdrg_op &o = next();
      if (o.kind == XDRG_OP_UNION) {
        const std::int32_t d = static_cast<std::int32_t>(f);
        std::memcpy(R() + o.noff, &d, 4);
        branch(o, d);
      } else {
        std::memcpy(R() + o.noff, &f, sizeof(P));
        ++pc;
      }
    } else if constexpr (vector_info<P>::value) {
      const xdrg_op &o = next();
      const std::uint32_t cnt = static_cast<std::uint32_t>(f.size());
      heap->resize((heap->size() + 7) & ~std::size_t(7), 0);
      const std::uint64_t off = heap->size();
      heap->resize(off + std::uint64_t(cnt) * o.arg1, 0);
      const std::uint32_t entry = (o.flags & XDRG_F_SUB) ? o.arg4 : pc + 1;
      std::uint32_t i = 0;
      for (const auto &e : f) {
        stager<V> s2;
        s2.ops = ops;
        s2.table = table;
        s2.pc = entry;
        s2.heap = heap;
        s2.in_heap = true;
        s2.roff = off + std::uint64_t(i++) * o.arg1;
        s2(e);
      }
      const xdrg_bytes_ref r{off, cnt, 0};
      std::memcpy(R() + o.noff, &r, sizeof r);
      pc += 1 + o.arg2;
    } else if constexpr (xarray_info<P>::value) {
      for (const auto &e : f) (*this)(e);
    } else {
      TR::save(*this, f);
    }
  }
};

// Thrown by an unstager that reaches its stop op (the op a device decode
// failed at): the caller raises the device's error there.
struct stop_reached {};
constexpr std::uint32_t kNoStop = 0xffffffffu;

// Unstage: xdr_traits<T>::load reads the staged record back, so every
// struct and union ends with its validate() hook, in the reference's order.
// With `stop` set, the walk throws stop_reached on reaching that op: the
// hooks of everything decoded before it have run, as they would have in
// xdr_generic_get before the failing field.
// Does the failure of a decoded object (walked from pc) lie inside one of
// its element subroutines?  Those containers carry rsv = 1 + the failing
// element (xdrgpu.h); the walk follows the object's own discriminants.
inline bool failure_deeper(const xdrg_op *ops, const std::uint32_t *table, const std::uint8_t *rec,
                           std::uint32_t pc) {
  for (;;) {
    const xdrg_op &o = ops[pc];
    switch (o.kind) {
    case XDRG_OP_END: return false;
    case XDRG_OP_JUMP: pc = o.arg0; break;
    case XDRG_OP_UNION: {
      std::int32_t d;
      std::memcpy(&d, rec + o.noff, 4);
      cursor c{ops, table, pc};
      try { c.branch(o, d); } catch (const xdr_bad_discriminant &) { return false; }
      pc = c.pc;
      break;
    }
    case XDRG_OP_VECTOR: {
      xdrg_bytes_ref r;
      std::memcpy(&r, rec + o.noff, sizeof r);
      if ((o.flags & XDRG_F_SUB) && r.rsv) return true;
      pc += 1 + o.arg2;
      break;
    }
    default: ++pc; break;
    }
  }
}

struct unstager : cursor {
  const std::uint8_t *rec;
  const std::uint8_t *heap;
  std::uint32_t stop = kNoStop;
  bool here = true;  // the stop op is in this object's own walk, not in an element's
  void at_op() const {
    if (pc == stop && here) throw stop_reached{};
  }
  template <typename F> void operator()(F &f) {
    using P = plain<F>;
    using TR = xdr_traits<P>;
    if constexpr (std::is_same_v<P, bool>) {
      f = rec[next().noff] != 0;
      at_op();
      ++pc;
    } else if constexpr (bytes_kind<P>::kind == XDRG_OP_OPAQUE) {
      const xdrg_op &o = next();
      at_op();
      std::memcpy(f.data(), rec + o.noff, f.size());
      ++pc;
    } else if constexpr (bytes_kind<P>::kind != 0) {
      const xdrg_op &o = next();
      at_op();
      xdrg_bytes_ref r;
      std::memcpy(&r, rec + o.noff, sizeof r);
      const char *p = reinterpret_cast<const char *>(heap + r.off);
      f.assign(p, p + r.len);
      ++pc;
    } else if constexpr (TR::is_enum || TR::is_numeric) {
      const xdrg_op &o = next();
      at_op();
      std::memcpy(&f, rec + o.noff, sizeof(P));
      if (o.kind == XDRG_OP_UNION) branch(o, static_cast<std::int32_t>(f));
      else ++pc;
    } else if constexpr (vector_info<P>::value) {
      const xdrg_op &o = next();
      at_op();
      xdrg_bytes_ref r;
      std::memcpy(&r, rec + o.noff, sizeof r);
      // A decode that failed inside an element decoded the ones before it:
      // inline (fixed) elements when the failing op is one of theirs
      // (rsv = the failing element), subroutine elements on the marked
      // path (rsv = 1 + the failing element).
      const bool sub = (o.flags & XDRG_F_SUB) != 0;
      const bool inside = stop != kNoStop &&
                          (sub ? r.rsv != 0 : here && stop > pc && stop <= pc + o.arg2);
      const std::uint32_t whole = !inside ? r.len : std::min(sub ? r.rsv - 1 : r.rsv, r.len);
      const std::uint32_t entry = sub ? o.arg4 : pc + 1;
      if constexpr (vector_info<P>::pointer) {
        if (r.len) f.activate(); else f.reset();
      } else {
        f.resize(r.len);
      }
      std::uint32_t i = 0;
      for (auto &e : f) {
        if (i > whole || (i == whole && !inside)) break;
        unstager u2;
        u2.ops = ops;
        u2.table = table;
        u2.pc = entry;
        u2.rec = heap + r.off + std::uint64_t(i) * o.arg1;
        u2.heap = heap;
        if (i == whole) {
          u2.stop = stop;
          u2.here = !sub || !failure_deeper(ops, table, u2.rec, entry);
        }
        u2(e);
        ++i;
      }
      if (inside) throw stop_reached{};
      pc += 1 + o.arg2;
    } else if constexpr (xarray_info<P>::value) {
      for (auto &e : f) (*this)(e);
    } else {
      TR::load(*this, f);
    }
  }
};

inline std::uint32_t be32(const std::uint8_t *p) {
  return (std::uint32_t(p[0]) << 24) | (std::uint32_t(p[1]) << 16) | (std::uint32_t(p[2]) << 8) | p[3];
}

inline void hipcheck(hipError_t e, const char *what) {
  if (e != hipSuccess) throw api_error(XDRG_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
inline void abicheck(int rc, const char *what) {
  if (rc != XDRG_OK) {
    const char *h = xdrg_last_hip_error();
    throw api_error(rc, std::string(what) + " failed (" + std::to_string(rc) + ")" +
                            (rc == XDRG_EHIP && h ? std::string(": ") + h : std::string()));
  }
}

//! A device buffer that only grows: reused from call to call.
struct grow_buf {
  void *p = nullptr;
  std::size_t cap = 0;
  template <typename T> T *get(std::size_t n) {
    const std::size_t bytes = std::max<std::size_t>(n * sizeof(T), 16);
    if (bytes > cap) {
      if (p) hipcheck(hipFree(p), "hipFree");  // hipFree waits for the work using it
      p = nullptr;
      cap = 0;
      hipcheck(hipMalloc(&p, bytes), "hipMalloc");
      ++alloc_count();
      cap = bytes;
    }
    return static_cast<T *>(p);
  }
  grow_buf() = default;
  grow_buf(const grow_buf &) = delete;
  grow_buf &operator=(const grow_buf &) = delete;
  ~grow_buf() { if (p) (void)hipFree(p); }
};

}  // namespace detail

// ---------------------------------------------------------------- the plan
//! The device plan of T (built once, thread-safe).
template <typename T> class batch_plan {
 public:
  static const batch_plan &get() {
    static const batch_plan p;
    return p;
  }
  xdrg_plan *handle() const { return h_.get(); }
  const std::vector<xdrg_op> &ops() const { return ops_; }
  const std::vector<std::uint32_t> &table() const { return table_; }
  std::uint32_t stride() const { return stride_; }
  //! Records are passed to the device as-is (staged layout == C++ layout).
  bool identity() const { return identity_; }
  bool fixed() const { return fixed_; }
  std::uint32_t fixed_size() const { return fixed_size_; }
  //! Largest wire record the plan's bounds allow (all-ones: unbounded).
  std::uint64_t max_record_bytes() const { return max_record_bytes_; }
  //! Some struct or union of T has a user validate() hook.
  bool validates() const { return validates_; }

  //! Throw the reference's exception for a device status.
  [[noreturn]] void raise(const xdrg_error &e) const {
    std::string what = xdrg_error_message(e.code);
    if (e.code == XDRG_ERR_BAD_DISCRIMINANT)
      for (const auto &m : msgs_)
        if (m.first == e.op) what = m.second;
    switch (xdrg_error_exception(e.code)) {
    case XDRG_EXC_OVERFLOW: throw xdr_overflow(what);
    case XDRG_EXC_STACK_OVERFLOW: throw xdr_stack_overflow(what);
    case XDRG_EXC_BAD_MESSAGE_SIZE: throw xdr_bad_message_size(what);
    case XDRG_EXC_BAD_DISCRIMINANT: throw xdr_bad_discriminant(what);
    case XDRG_EXC_SHOULD_BE_ZERO: throw xdr_should_be_zero(what);
    case XDRG_EXC_INVARIANT_FAILED: throw xdr_invariant_failed(what);
    default: throw xdr_runtime_error(what);
    }
  }

 private:
  struct deleter { void operator()(xdrg_plan *p) const { xdrg_plan_destroy(p); } };
  batch_plan() {
    if constexpr (detail::has_emitted_plan<T>::value) {
      using E = emitted_plan<T>;
      ops_.assign(E::ops, E::ops + E::nops);
      table_.assign(E::table, E::table + E::ntable);
      msgs_ = E::msgs();
      stride_ = E::stride;
      // xdrc's C++ type of a fixed-size record is laid out as the plan stages
      // it (natural alignment, bool 1 byte, enums 4) when its size agrees
      identity_ = E::fixed && std::is_trivially_copyable_v<T> && sizeof(T) == stride_;
      fixed_ = E::fixed;
      validates_ = E::validates;
      create(E::kernels);
    } else {
      record();
      create("");
    }
  }
  // the plan from the tables, and the emitted code object when there is one
  void create(const char *kernels) {
    xdrg_plan *h = nullptr;
    detail::abicheck(xdrg_plan_create(ops_.data(), static_cast<std::uint32_t>(ops_.size()),
                                      table_.empty() ? nullptr : table_.data(),
                                      static_cast<std::uint32_t>(table_.size()), stride_, &h),
                     "xdrg_plan_create");
    h_.reset(h);
    if (kernels && *kernels) {
      const char *dir = std::getenv("XDRG_PLAN_KERNEL_DIR");
#ifdef XDRG_EMITTED_KERNEL_DIR
      if (!dir) dir = XDRG_EMITTED_KERNEL_DIR;
#endif
      if (dir) {
        const std::string path = std::string(dir) + "/" + kernels + ".co";
        if (FILE *f = std::fopen(path.c_str(), "rb")) {
          std::vector<char> co;
          char buf[1 << 16];
          for (std::size_t k; (k = std::fread(buf, 1, sizeof buf, f)) > 0;) co.insert(co.end(), buf, buf + k);
          std::fclose(f);
          detail::abicheck(xdrg_plan_load_kernels(h, co.data(), co.size()), "xdrg_plan_load_kernels");
        }
      }
    }
    xdrg_plan_info info{};
    detail::abicheck(xdrg_plan_get_info(h, &info), "xdrg_plan_get_info");
    fixed_size_ = info.fixed_size;
    max_record_bytes_ = info.max_record_bytes;
  }
  // the plan recorded from xdr_traits<T>
  void record() {
    ++detail::recorded_plans();
    // the record's ops, END, then one element subroutine per element type
    // (each ending with END); F_SUB VECTOR ops get the body's stride and pc
    detail::sub_registry subs;
    subs.types.push_back(std::type_index(typeid(T)));  // key 0: the record's own ops (pc 0)
    subs.bodies.emplace_back();
    detail::sub_registry *outer = detail::active_subs();
    detail::active_subs() = &subs;
    detail::subplan sp;
    try {
      sp = detail::record_type<T>();
    } catch (...) {
      detail::active_subs() = outer;
      throw;
    }
    detail::active_subs() = outer;
    subs.bodies[0] = sp;
    detail::subplan top;
    detail::append(top, sp, 0, 0);
    top.ops.push_back(detail::mkop(XDRG_OP_END, 0, 0));
    // bodies in order of first reference, breadth first from the record
    // (the order xdrpp_amd/xdr_types.py emits them in)
    const std::size_t nk = subs.bodies.size();
    std::vector<std::uint32_t> entry(nk, 0xffffffffu), order;
    entry[0] = 0;
    auto refs = [&](const detail::subplan &b) {
      for (const xdrg_op &o : b.ops)
        if (o.kind == XDRG_OP_VECTOR && (o.flags & XDRG_F_SUB) && entry[o.arg4] == 0xffffffffu) {
          entry[o.arg4] = 0;  // queued
          order.push_back(o.arg4);
        }
    };
    refs(sp);
    bool validates = sp.validates;
    for (std::size_t q = 0; q < order.size(); ++q) {
      const std::uint32_t k = order[q];
      entry[k] = static_cast<std::uint32_t>(top.ops.size());
      detail::append(top, subs.bodies[k], 0, 0);
      top.ops.push_back(detail::mkop(XDRG_OP_END, 0, 0));
      validates = validates || subs.bodies[k].validates;
      refs(subs.bodies[k]);
    }
    for (xdrg_op &o : top.ops)
      if (o.kind == XDRG_OP_VECTOR && (o.flags & XDRG_F_SUB)) {
        const detail::subplan &b = subs.bodies[o.arg4];
        o.arg1 = detail::align_up(std::max<std::uint32_t>(b.size, 1), b.align);
        o.arg4 = entry[o.arg4];
      }
    ops_ = std::move(top.ops);
    table_ = std::move(top.table);
    msgs_ = std::move(top.msgs);
    stride_ = detail::align_up(std::max<std::uint32_t>(sp.size, 1), std::max<std::uint32_t>(sp.align, 4));
    identity_ = sp.identity && sp.fixed && sizeof(T) == stride_;
    fixed_ = sp.fixed;
    validates_ = validates;
  }
  struct record_only {};
  explicit batch_plan(record_only) { record(); }
  template <typename U> friend struct recorded_plan;
  std::unique_ptr<xdrg_plan, deleter> h_;
  std::vector<xdrg_op> ops_;
  std::vector<std::uint32_t> table_;
  std::vector<std::pair<std::uint32_t, std::string>> msgs_;
  std::uint32_t stride_ = 0, fixed_size_ = 0;
  std::uint64_t max_record_bytes_ = 0;
  bool identity_ = false, fixed_ = false, validates_ = false;
};

template <typename T> const batch_plan<T> &plan_for() { return batch_plan<T>::get(); }

//! The plan recorded from xdr_traits<T>, whether or not T has an emitted
//! one (tests compare the two op for op).
template <typename T> struct recorded_plan {
  std::vector<xdrg_op> ops;
  std::vector<std::uint32_t> table;
  std::vector<std::pair<std::uint32_t, std::string>> msgs;
  std::uint32_t stride = 0;
  bool identity = false, fixed = false, validates = false;
  recorded_plan() {
    const batch_plan<T> r{typename batch_plan<T>::record_only{}};
    ops = r.ops_;
    table = r.table_;
    msgs = r.msgs_;
    stride = r.stride_;
    identity = r.identity_;
    fixed = r.fixed_;
    validates = r.validates_;
  }
};

// ---------------------------------------------------------------- staging
//! Host staging of a batch: records in the staged layout + payload heap.
//! (A context stages into pinned memory, so that the copies to the device
//! run asynchronously.)
template <typename A = std::allocator<std::uint8_t>> struct basic_staged_batch {
  std::vector<std::uint8_t, A> native;
  std::vector<std::uint8_t, A> heap;
};
using staged_batch = basic_staged_batch<>;

//! Stage n records into b, reusing its buffers' capacity.
template <typename T, typename A> void stage_into(basic_staged_batch<A> &b, const T *recs, std::size_t n) {
  const batch_plan<T> &P = plan_for<T>();
  b.native.assign(n * P.stride(), 0);
  b.heap.clear();
  if (P.identity()) {
    if (n) std::memcpy(b.native.data(), recs, n * sizeof(T));
    return;
  }
  for (std::size_t i = 0; i < n; ++i) {
    detail::stager<std::vector<std::uint8_t, A>> s;
    s.ops = P.ops().data();
    s.table = P.table().data();
    s.rec = b.native.data() + i * P.stride();
    s.heap = &b.heap;
    s(recs[i]);
  }
}

template <typename T> staged_batch stage(const T *recs, std::size_t n) {
  staged_batch b;
  stage_into(b, recs, n);
  return b;
}

//! The buffers of the batch calls -- device buffers and pinned host staging
//! that only grow, so a context serving batches of a steady size allocates
//! nothing after its first call -- used by one thread at a time.  The
//! calls that take no context use their thread's default one (per device).
class context {
 public:
  context() = default;
  context(const context &) = delete;
  context &operator=(const context &) = delete;
  //! Device and pinned buffers allocated so far by every context.
  static std::size_t allocations() { return detail::alloc_count(); }

  // device buffers
  detail::grow_buf d_nat, d_heap, d_xdr, d_off, d_ws, d_st, d_aux, d_cnt;
  // pinned host staging
  basic_staged_batch<detail::pinned_allocator<std::uint8_t>> staged;
  detail::host_bytes h_in, h_out, h_heap, h_off;
  xdrg_status *status() { return d_st.get<xdrg_status>(1); }
};

//! The calling thread's default context on the current device.  (Never
//! destroyed: its buffers must not be freed after the HIP runtime's own
//! teardown at exit.)
inline context &default_context() {
  thread_local std::vector<context *> per_device;
  int d = 0;
  detail::hipcheck(hipGetDevice(&d), "hipGetDevice");
  if (per_device.size() <= static_cast<std::size_t>(d)) per_device.resize(d + 1, nullptr);
  if (!per_device[d]) per_device[d] = new context();
  return *per_device[d];
}

namespace detail {
//! H2D of a staged batch into the context's device buffers.
inline void upload(context &c, hipStream_t s, std::uint8_t **nat, std::uint8_t **heap) {
  *nat = c.d_nat.get<std::uint8_t>(c.staged.native.size());
  *heap = c.staged.heap.empty() ? nullptr : c.d_heap.get<std::uint8_t>(c.staged.heap.size());
  if (!c.staged.native.empty())
    hipcheck(hipMemcpyAsync(*nat, c.staged.native.data(), c.staged.native.size(), hipMemcpyHostToDevice, s), "H2D");
  if (*heap)
    hipcheck(hipMemcpyAsync(*heap, c.staged.heap.data(), c.staged.heap.size(), hipMemcpyHostToDevice, s), "H2D");
}
//! Stage host bytes into pinned memory and copy them to a device buffer.
inline std::uint8_t *upload_bytes(context &c, grow_buf &d, const void *bytes, std::size_t len, hipStream_t s) {
  std::uint8_t *p = d.get<std::uint8_t>(len);
  if (len) {
    c.h_in.resize(len);
    std::memcpy(c.h_in.data(), bytes, len);
    hipcheck(hipMemcpyAsync(p, c.h_in.data(), len, hipMemcpyHostToDevice, s), "H2D");
  }
  return p;
}
}  // namespace detail

template <typename T>
void unstage(const std::uint8_t *native, const std::uint8_t *heap, std::size_t n, T *out) {
  const batch_plan<T> &P = plan_for<T>();
  if (P.identity() && !P.validates()) {
    std::memcpy(static_cast<void *>(out), native, n * sizeof(T));
    return;
  }
  for (std::size_t i = 0; i < n; ++i) {
    detail::unstager u;
    u.ops = P.ops().data();
    u.table = P.table().data();
    u.rec = native + i * P.stride();
    u.heap = heap;
    u(out[i]);
  }
}

//! The records of a device decode whose status is `e`, in the order
//! xdr_from_opaque / xdr_from_msg would load them: records before the
//! failing one are unstaged in full (their validate() hooks run and the
//! first hook that throws wins, xdrc/gen_hh.cc:244-247), then the failing
//! record up to the op the device failed at, then the device's error is
//! raised.  A record-level error (op 0xffffffff) at record r < n raises
//! before record r; one at record n (trailing bytes, seen by done() after
//! every record loaded) raises after all of them.
template <typename T>
void unstage_checked(const std::uint8_t *native, const std::uint8_t *heap, std::size_t n, T *out,
                     const xdrg_error &e) {
  const batch_plan<T> &P = plan_for<T>();
  if (!e.code) {
    unstage(native, heap, n, out);
    return;
  }
  const std::size_t bad = static_cast<std::size_t>(std::min<std::uint64_t>(e.record, n));
  if (P.validates()) {
    unstage(native, heap, bad, out);
    if (bad < n && e.op != 0xffffffffu) {
      detail::unstager u;
      u.ops = P.ops().data();
      u.table = P.table().data();
      u.rec = native + bad * P.stride();
      u.heap = heap;
      u.stop = e.op;
      u.here = !detail::failure_deeper(u.ops, u.table, u.rec, 0);
      try {
        u(out[bad]);
      } catch (const detail::stop_reached &) {
      }
    }
  }
  P.raise(e);
}

//! Record index of a concatenated batch (host walk of lengths and
//! discriminants only).  Records that would overrun `len` or carry a bad
//! discriminant end the walk; the remaining offsets are `len`, and the
//! device decode then reports the reference's error for that record.
namespace detail {
// Step p over one object's wire bytes (the walk from pc to its END): false
// when the bytes run out or a discriminant is bad.  Element subroutines are
// walked with an explicit stack, so nesting is bounded by the bytes only
// (every element consumes at least 4 of them).
inline bool skip_object(const xdrg_op *ops, const std::uint32_t *tab, const std::uint8_t *xdr,
                        std::size_t len, std::uint64_t &p, std::uint32_t pc) {
  struct frame {
    std::uint32_t left, vpc;  // elements after the current one; the VECTOR op
  };
  std::vector<frame> st;
  for (;;) {
    const xdrg_op &o = ops[pc];
    switch (o.kind) {
    case XDRG_OP_END:
      if (st.empty()) return true;
      if (st.back().left) {
        --st.back().left;
        pc = ops[st.back().vpc].arg4;
        if (p > len) return false;
      } else {
        pc = st.back().vpc + 1;
        st.pop_back();
      }
      continue;
    case XDRG_OP_JUMP: pc = o.arg0; continue;
    case XDRG_OP_U64: p += 8; break;
    case XDRG_OP_OPAQUE: p += align_up(o.arg0, 4); break;
    case XDRG_OP_VAROPAQUE: case XDRG_OP_STRING:
      if (p + 4 > len) return false;
      p += 4 + ((std::uint64_t(be32(xdr + p)) + 3) & ~3ull);
      break;
    case XDRG_OP_VECTOR: {
      if (p + 4 > len) return false;
      const std::uint32_t cnt = be32(xdr + p);
      p += 4;
      if (o.flags & XDRG_F_SUB) {
        if (cnt) {
          if (p > len) return false;
          st.push_back(frame{cnt - 1, pc});
          pc = o.arg4;
        } else {
          ++pc;
        }
        continue;
      }
      std::uint64_t we = 0;
      for (std::uint32_t k = 1; k <= o.arg2; ++k) {
        const xdrg_op &e = ops[pc + k];
        we += e.kind == XDRG_OP_U64 ? 8u : e.kind == XDRG_OP_OPAQUE ? align_up(e.arg0, 4) : 4u;
      }
      p += cnt * we;
      pc += 1 + o.arg2;
      continue;
    }
    case XDRG_OP_UNION: {
      if (p + 4 > len) return false;
      const std::int32_t d = static_cast<std::int32_t>(be32(xdr + p));
      p += 4;
      cursor c{ops, tab, pc};
      try { c.branch(o, d); } catch (const xdr_bad_discriminant &) { return false; }
      pc = c.pc;
      continue;
    }
    default: p += 4; break;
    }
    ++pc;
  }
}
}  // namespace detail

template <typename T>
std::vector<std::uint64_t> index_records(const std::uint8_t *xdr, std::size_t len, std::size_t n) {
  const batch_plan<T> &P = plan_for<T>();
  std::vector<std::uint64_t> off(n + 1, len);
  std::uint64_t p = 0;
  for (std::size_t r = 0; r < n; ++r) {
    off[r] = std::min<std::uint64_t>(p, len);
    if (!detail::skip_object(P.ops().data(), P.table().data(), xdr, len, p, 0) || p > len)
      return off;  // off[r] is set; the rest stay at len
  }
  off[n] = p;  // p < len: trailing bytes, which decode reports at record n
  return off;
}

// ------------------------------------------------------------ batch calls
namespace detail {
//! Read the status block (waits for the stream); raise on a data error.
template <typename T> xdrg_error read_status(context &c, hipStream_t s, bool raise_it = true) {
  xdrg_error e{};
  abicheck(xdrg_status_read(c.status(), s, &e), "xdrg_status_read");
  if (raise_it && e.code) plan_for<T>().raise(e);
  return e;
}

//! The batch encoded on the device: the context's d_xdr holds `total`
//! bytes, d_off the record (msgs: message) offsets.  One size pass: the
//! output is sized by xdrg_encode_sizes, as xdr_to_opaque sizes the
//! argument pack (marshal.h:264-268), and xdrg_encode_sized encodes over it.
template <typename T> std::size_t encode_on_device(context &c, const T *recs, std::size_t n, bool msgs,
                                                   hipStream_t s) {
  const batch_plan<T> &P = plan_for<T>();
  stage_into(c.staged, recs, n);
  std::uint8_t *nat = nullptr, *heap = nullptr;
  upload(c, s, &nat, &heap);
  const std::size_t hl = c.staged.heap.size();
  abicheck(xdrg_status_init(c.status(), s), "xdrg_status_init");
  const std::size_t ws_bytes = xdrg_workspace_size(P.handle(), n);
  void *ws = c.d_ws.get<std::uint8_t>(ws_bytes);
  std::uint64_t *off = c.d_off.get<std::uint64_t>(n + 1);
  std::size_t total = (std::size_t(P.fixed_size()) + (msgs ? 4 : 0)) * n;
  if (!P.fixed() || msgs) {
    abicheck(xdrg_encode_sizes(P.handle(), nat, n, heap, hl, marshaling_stack_limit, msgs, ws, ws_bytes,
                               c.status(), s),
             "xdrg_encode_sizes");
    total = read_status<T>(c, s).total_bytes;
  }
  std::uint8_t *out = c.d_xdr.get<std::uint8_t>(total);
  abicheck(xdrg_encode_sized(P.handle(), nat, n, heap, hl, out, total, (P.fixed() && !msgs) ? nullptr : off,
                             marshaling_stack_limit, msgs, ws, ws_bytes, c.status(), s),
           "xdrg_encode_sized");
  return total;
}
}  // namespace detail

//! xdr::xdr_to_opaque(recs[0], ..., recs[n-1]) on the GPU.  Host in, host
//! out, through the context's pinned staging (the device-resident entry
//! point is xdrg_encode).
template <typename T>
opaque_vec<> to_opaque_batch(context &c, const T *recs, std::size_t n, hipStream_t s = nullptr) {
  const std::size_t total = detail::encode_on_device(c, recs, n, false, s);
  c.h_out.resize(total);
  if (total)
    detail::hipcheck(hipMemcpyAsync(c.h_out.data(), c.d_xdr.p, total, hipMemcpyDeviceToHost, s), "D2H");
  detail::read_status<T>(c, s);
  opaque_vec<> out;
  out.resize(total);
  if (total) std::memcpy(out.data(), c.h_out.data(), total);
  return out;
}
template <typename T>
opaque_vec<> to_opaque_batch(const T *recs, std::size_t n, hipStream_t s = nullptr) {
  return to_opaque_batch(default_context(), recs, n, s);
}

//! xdr::xdr_from_opaque(bytes, out[0], ..., out[n-1]) on the GPU.
template <typename T>
void from_opaque_batch(context &c, const void *bytes, std::size_t len, T *out, std::size_t n,
                       hipStream_t s = nullptr) {
  const batch_plan<T> &P = plan_for<T>();
  const auto *x = static_cast<const std::uint8_t *>(bytes);
  std::uint8_t *d_x = detail::upload_bytes(c, c.d_xdr, x, len, s);
  std::uint8_t *d_nat = c.d_nat.get<std::uint8_t>(n * P.stride());
  detail::abicheck(xdrg_status_init(c.status(), s), "xdrg_status_init");
  std::uint64_t *d_off = P.fixed() ? nullptr : c.d_off.get<std::uint64_t>(n + 1);
  const std::uint64_t hcap = P.fixed() ? 0 : xdrg_decode_heap_size(P.handle(), len);
  std::uint8_t *d_heap = hcap ? c.d_heap.get<std::uint8_t>(hcap) : nullptr;
  if (!P.fixed()) {
    // the record index on the device (xdrg_index_records): records of any
    // length and nesting (longer ones than the index window are walked on
    // the device between list-ranking windows); a plan the index cannot
    // chain (records under 4 bytes) is walked on the host
    std::uint32_t win = static_cast<std::uint32_t>(
        std::min<std::uint64_t>(std::max<std::uint64_t>(P.max_record_bytes(), 16), XDRG_MAX_MSG));
    std::uint64_t *d_cnt = c.d_cnt.get<std::uint64_t>(1);
    int rc = XDRG_OK;
    for (;;) {
      const std::size_t wsb = xdrg_index_workspace_size(len, win);
      void *ws = c.d_ws.get<std::uint8_t>(wsb);
      rc = xdrg_index_records(P.handle(), d_x, len, n, win, d_off, d_cnt, ws, wsb, c.status(), s);
      if (rc == XDRG_EUNSUPPORTED) break;
      detail::abicheck(rc, "xdrg_index_records");
      const xdrg_error ie = detail::read_status<T>(c, s, false);
      if (ie.code == XDRG_ERR_INDEX_LONG && win <= XDRG_INDEX_MAX_MSG) {
        // a record nested past the window parse's frames, or longer than
        // the plan's bound: the whole-stream walk (no length bound, nesting
        // to XDRG_MAX_FRAMES), and the decode reports the record's own error
        win = XDRG_MAX_MSG;
        detail::abicheck(xdrg_status_init(c.status(), s), "xdrg_status_init");
        continue;
      }
      if (ie.code) P.raise(ie);
      break;
    }
    const bool host = rc == XDRG_EUNSUPPORTED;
    if (host) {
      const std::vector<std::uint64_t> idx = index_records<T>(x, len, n);
      c.h_off.resize((n + 1) * 8);
      std::memcpy(c.h_off.data(), idx.data(), (n + 1) * 8);
      detail::hipcheck(hipMemcpyAsync(d_off, c.h_off.data(), (n + 1) * 8, hipMemcpyHostToDevice, s), "H2D");
    }
  }
  const std::size_t dws = xdrg_deep_workspace_size(P.handle(), n);  // deep plans' passes
  void *dw = dws ? c.d_ws.get<std::uint8_t>(dws) : nullptr;
  detail::abicheck(xdrg_decode(P.handle(), d_x, len, d_off, n, d_nat, d_heap, hcap, marshaling_stack_limit,
                               dw, dws, c.status(), s),
                   "xdrg_decode");
  c.h_out.resize(n * P.stride());
  c.h_heap.resize(hcap);
  if (!c.h_out.empty())
    detail::hipcheck(hipMemcpyAsync(c.h_out.data(), d_nat, c.h_out.size(), hipMemcpyDeviceToHost, s), "D2H");
  if (hcap) detail::hipcheck(hipMemcpyAsync(c.h_heap.data(), d_heap, hcap, hipMemcpyDeviceToHost, s), "D2H");
  const xdrg_error e = detail::read_status<T>(c, s, false);
  unstage_checked(c.h_out.data(), c.h_heap.data(), n, out, e);
}
template <typename T>
void from_opaque_batch(const void *bytes, std::size_t len, T *out, std::size_t n, hipStream_t s = nullptr) {
  from_opaque_batch(default_context(), bytes, len, out, n, s);
}

// ------------------------------------------------------ sizes and depths
//! xdr::xdr_size(recs[i]) for every record (xdrpp/types.h:240-244), one
//! device size pass (xdrg_serial_sizes).
template <typename T>
std::vector<std::uint32_t> xdr_size_batch(context &c, const T *recs, std::size_t n, hipStream_t s = nullptr) {
  const batch_plan<T> &P = plan_for<T>();
  stage_into(c.staged, recs, n);
  std::uint8_t *nat = nullptr, *heap = nullptr;
  detail::upload(c, s, &nat, &heap);
  std::uint32_t *d_sz = c.d_aux.get<std::uint32_t>(n);
  detail::abicheck(xdrg_status_init(c.status(), s), "xdrg_status_init");
  const std::size_t dws = xdrg_deep_workspace_size(P.handle(), n);
  void *dw = dws ? c.d_ws.get<std::uint8_t>(dws) : nullptr;
  detail::abicheck(xdrg_serial_sizes(P.handle(), nat, n, heap, c.staged.heap.size(), d_sz, marshaling_stack_limit,
                                     dw, dws, c.status(), s),
                   "xdrg_serial_sizes");
  c.h_out.resize(n * 4);
  if (n) detail::hipcheck(hipMemcpyAsync(c.h_out.data(), d_sz, n * 4, hipMemcpyDeviceToHost, s), "D2H");
  detail::read_status<T>(c, s);
  std::vector<std::uint32_t> out(n);
  if (n) std::memcpy(out.data(), c.h_out.data(), n * 4);
  return out;
}
template <typename T>
std::vector<std::uint32_t> xdr_size_batch(const T *recs, std::size_t n, hipStream_t s = nullptr) {
  return xdr_size_batch(default_context(), recs, n, s);
}

//! xdr::check_xdr_depth(recs[i], depth_limit) for every record
//! (xdrpp/depth_checker.h:72-79), from the device's per-record depths
//! (xdrg_record_depths).
template <typename T>
std::vector<bool> check_xdr_depth_batch(context &c, const T *recs, std::size_t n, std::uint32_t depth_limit,
                                        hipStream_t s = nullptr) {
  const batch_plan<T> &P = plan_for<T>();
  stage_into(c.staged, recs, n);
  std::uint8_t *nat = nullptr, *heap = nullptr;
  detail::upload(c, s, &nat, &heap);
  std::uint32_t *d_d = c.d_aux.get<std::uint32_t>(n);
  detail::abicheck(xdrg_status_init(c.status(), s), "xdrg_status_init");
  const std::size_t dws = xdrg_deep_workspace_size(P.handle(), n);
  void *dw = dws ? c.d_ws.get<std::uint8_t>(dws) : nullptr;
  detail::abicheck(xdrg_record_depths(P.handle(), nat, n, heap, c.staged.heap.size(), d_d, dw, dws, c.status(), s),
                   "xdrg_record_depths");
  c.h_out.resize(n * 4);
  if (n) detail::hipcheck(hipMemcpyAsync(c.h_out.data(), d_d, n * 4, hipMemcpyDeviceToHost, s), "D2H");
  detail::read_status<T>(c, s);
  std::vector<bool> ok(n);
  for (std::size_t i = 0; i < n; ++i) {
    std::uint32_t d;
    std::memcpy(&d, c.h_out.data() + 4 * i, 4);
    ok[i] = d <= depth_limit;
  }
  return ok;
}
template <typename T>
std::vector<bool> check_xdr_depth_batch(const T *recs, std::size_t n, std::uint32_t depth_limit,
                                        hipStream_t s = nullptr) {
  return check_xdr_depth_batch(default_context(), recs, n, depth_limit, s);
}

// ---------------------------------------------------- record-marked messages
namespace detail {
// Device encode of n staged records as n record-marked messages.  Returns
// the stream and fills off[n+1] (mark of each message, then the total).
template <typename T>
std::vector<std::uint8_t> encode_msgs(context &c, const T *recs, std::size_t n, std::vector<std::uint64_t> &off,
                                      hipStream_t s) {
  const std::size_t total = encode_on_device(c, recs, n, true, s);
  c.h_out.resize(total);
  c.h_off.resize((n + 1) * 8);
  if (total) hipcheck(hipMemcpyAsync(c.h_out.data(), c.d_xdr.p, total, hipMemcpyDeviceToHost, s), "D2H");
  hipcheck(hipMemcpyAsync(c.h_off.data(), c.d_off.p, (n + 1) * 8, hipMemcpyDeviceToHost, s), "D2H");
  read_status<T>(c, s);
  off.assign(n + 1, 0);
  std::memcpy(off.data(), c.h_off.data(), (n + 1) * 8);
  return std::vector<std::uint8_t>(c.h_out.begin(), c.h_out.begin() + std::ptrdiff_t(total));
}

// Device decode of the n messages of a stream (already on the device at
// d_x) indexed by d_off.
template <typename T>
void decode_msgs_on_device(context &c, const std::uint8_t *d_x, std::size_t len, const std::uint64_t *d_off, T *out,
                           std::size_t n, hipStream_t s) {
  const batch_plan<T> &P = plan_for<T>();
  std::uint8_t *d_nat = c.d_nat.get<std::uint8_t>(n * P.stride());
  abicheck(xdrg_status_init(c.status(), s), "xdrg_status_init");
  const std::uint64_t hcap = P.fixed() ? 0 : xdrg_decode_heap_size(P.handle(), len);
  std::uint8_t *d_heap = hcap ? c.d_heap.get<std::uint8_t>(hcap) : nullptr;
  const std::size_t dws = xdrg_deep_workspace_size(P.handle(), n);  // deep plans' passes
  void *dw = dws ? c.d_ws.get<std::uint8_t>(dws) : nullptr;
  abicheck(xdrg_decode_msgs(P.handle(), d_x, len, d_off, n, d_nat, d_heap, hcap, marshaling_stack_limit, dw,
                            dws, c.status(), s),
           "xdrg_decode_msgs");
  c.h_out.resize(n * P.stride());
  c.h_heap.resize(hcap);
  if (!c.h_out.empty())
    hipcheck(hipMemcpyAsync(c.h_out.data(), d_nat, c.h_out.size(), hipMemcpyDeviceToHost, s), "D2H");
  if (hcap) hipcheck(hipMemcpyAsync(c.h_heap.data(), d_heap, hcap, hipMemcpyDeviceToHost, s), "D2H");
  const xdrg_error e = read_status<T>(c, s, false);
  unstage_checked(c.h_out.data(), c.h_heap.data(), n, out, e);
}

// The raw bytes (mark + body) of a vector of messages, back to back, into
// the context's pinned staging.
inline void concat(context &c, const std::vector<msg_ptr> &msgs, std::vector<std::uint64_t> &off) {
  off.assign(msgs.size() + 1, 0);
  for (std::size_t i = 0; i < msgs.size(); ++i) off[i + 1] = off[i] + msgs[i]->raw_size();
  c.h_in.resize(off.back());
  for (std::size_t i = 0; i < msgs.size(); ++i)
    std::memcpy(c.h_in.data() + off[i], msgs[i]->raw_data(), msgs[i]->raw_size());
}
}  // namespace detail

//! xdr::xdr_to_msg(recs[i]) for every record (marshal.h:252-260) in one
//! device pass: the messages back to back, as msg_sock::output writes a
//! queue of them (msgsock.cc:158-188).
template <typename T>
std::vector<std::uint8_t> to_msg_stream(const T *recs, std::size_t n, hipStream_t s = nullptr) {
  std::vector<std::uint64_t> off;
  return detail::encode_msgs(default_context(), recs, n, off, s);
}

//! The same messages, one message_t per record: msgs[i] holds the bytes
//! xdr::xdr_to_msg(recs[i]) produces (message_t::alloc, marshal.cc:15-31).
template <typename T>
std::vector<msg_ptr> to_msg_batch(const T *recs, std::size_t n, hipStream_t s = nullptr) {
  context &c = default_context();
  std::vector<std::uint64_t> off;
  detail::encode_msgs(c, recs, n, off, s);
  std::vector<msg_ptr> out;
  out.reserve(n);
  for (std::size_t i = 0; i < n; ++i) {
    msg_ptr m = message_t::alloc(off[i + 1] - off[i] - 4);
    std::memcpy(m->data(), c.h_out.data() + off[i] + 4, m->size());
    out.push_back(std::move(m));
  }
  return out;
}

//! xdr::xdr_from_msg(msgs[i], out[i]) for every message (marshal.h:278-284);
//! the first failing message raises the reference's exception.
template <typename T>
void from_msg_batch(const std::vector<msg_ptr> &msgs, T *out, hipStream_t s = nullptr) {
  context &c = default_context();
  std::vector<std::uint64_t> off;
  detail::concat(c, msgs, off);
  const std::size_t len = off.back(), n = msgs.size();
  std::uint8_t *d_x = c.d_xdr.get<std::uint8_t>(len);
  std::uint64_t *d_off = c.d_off.get<std::uint64_t>(n + 1);
  if (len) detail::hipcheck(hipMemcpyAsync(d_x, c.h_in.data(), len, hipMemcpyHostToDevice, s), "H2D");
  c.h_off.resize((n + 1) * 8);
  std::memcpy(c.h_off.data(), off.data(), (n + 1) * 8);
  detail::hipcheck(hipMemcpyAsync(d_off, c.h_off.data(), (n + 1) * 8, hipMemcpyHostToDevice, s), "H2D");
  detail::decode_msgs_on_device(c, d_x, len, d_off, out, n, s);
}

//! Every message of a stream of record-marked messages, decoded: the
//! framing of read_message / msg_sock::input (srpc.cc:29-55,
//! msgsock.cc:38-119) applied on the device (xdrg_index_msgs), messages of
//! up to max_msg_len bytes (msg_sock's default; any length up to 2^31 - 1),
//! then xdr_from_msg per message.  A framing error raises
//! xdr_bad_message_size.
template <typename T>
std::vector<T> from_msg_stream(const void *bytes, std::size_t len,
                               std::uint32_t max_msg_len = 0x100000,  // msg_sock::default_maxmsglen
                               hipStream_t s = nullptr) {
  context &c = default_context();
  const std::uint64_t max_msgs = len / 4;
  std::uint8_t *d_x = detail::upload_bytes(c, c.d_xdr, bytes, len, s);
  std::uint64_t *d_off = c.d_off.get<std::uint64_t>(max_msgs + 1);
  std::uint64_t *d_cnt = c.d_cnt.get<std::uint64_t>(1);
  const std::size_t ws_bytes = xdrg_index_workspace_size(len, max_msg_len);
  void *ws = c.d_ws.get<std::uint8_t>(ws_bytes);
  detail::abicheck(xdrg_status_init(c.status(), s), "xdrg_status_init");
  detail::abicheck(xdrg_index_msgs(d_x, len, max_msg_len, max_msgs, d_off, d_cnt, ws, ws_bytes, c.status(), s),
                   "xdrg_index_msgs");
  c.h_off.resize(8);
  detail::hipcheck(hipMemcpyAsync(c.h_off.data(), d_cnt, 8, hipMemcpyDeviceToHost, s), "D2H");
  xdrg_error e{};
  detail::abicheck(xdrg_status_read(c.status(), s, &e), "xdrg_status_read");
  if (e.code) throw xdr_bad_message_size(xdrg_error_message(e.code));
  std::uint64_t cnt = 0;
  std::memcpy(&cnt, c.h_off.data(), 8);
  std::vector<T> out(cnt);
  detail::decode_msgs_on_device(c, d_x, len, d_off, out.data(), cnt, s);
  return out;
}

// ------------------------------------------------------- RPC header batches
//! The procedures a server has registered: rpc_server_base::servers_
//! (server.h:218-219) with each interface's call_dispatch cases
//! (xdrc/gen_hh.cc:757-774), as the sorted table xdrg_rpc_dispatch takes.
class rpc_registry {
  std::vector<xdrg_rpc_proc> t_;

 public:
  //! register_service for (prog, vers) with these procedure numbers
  void add(std::uint32_t prog, std::uint32_t vers, const std::vector<std::uint32_t> &procs) {
    if (procs.empty()) t_.push_back({prog, vers, 0, XDRG_RPC_PROC_IFACE_ONLY});
    for (std::uint32_t p : procs) t_.push_back({prog, vers, p, 0});
    std::sort(t_.begin(), t_.end(), [](const xdrg_rpc_proc &a, const xdrg_rpc_proc &b) {
      return std::tie(a.prog, a.vers, a.proc) < std::tie(b.prog, b.vers, b.proc);
    });
    t_.erase(std::unique(t_.begin(), t_.end(),
                         [](const xdrg_rpc_proc &a, const xdrg_rpc_proc &b) {
                           return a.prog == b.prog && a.vers == b.vers && a.proc == b.proc;
                         }),
             t_.end());
    if (t_.size() > XDRG_RPC_MAX_PROCS) throw std::length_error("rpc_registry: too many procedures");
  }
  const std::vector<xdrg_rpc_proc> &table() const { return t_; }
};

//! rpc_server_base::dispatch's header decode and routing (server.cc:78-117)
//! for a batch of received messages, on the device.  hdrs[i].body_off and
//! .end are rebased to offsets into msgs[i]->data(), so the arguments of a
//! DISPATCH message decode with xdr_get(m->data() + body_off, m->end()).
inline std::vector<xdrg_rpc_hdr> rpc_dispatch_batch(const std::vector<msg_ptr> &msgs,
                                                    const rpc_registry &reg,
                                                    hipStream_t s = nullptr) {
  context &c = default_context();
  std::vector<std::uint64_t> off;
  detail::concat(c, msgs, off);
  const std::size_t n = msgs.size(), len = off.back(), np = reg.table().size();
  std::vector<xdrg_rpc_hdr> h(n);
  if (!n) return h;
  std::uint8_t *d_x = c.d_xdr.get<std::uint8_t>(len);
  std::uint64_t *d_off = c.d_off.get<std::uint64_t>(n + 1);
  xdrg_rpc_proc *d_p = c.d_aux.get<xdrg_rpc_proc>(np);
  xdrg_rpc_hdr *d_h = c.d_nat.get<xdrg_rpc_hdr>(n);
  c.h_off.resize((n + 1) * 8 + np * sizeof(xdrg_rpc_proc));
  std::memcpy(c.h_off.data(), off.data(), (n + 1) * 8);
  if (np) std::memcpy(c.h_off.data() + (n + 1) * 8, reg.table().data(), np * sizeof(xdrg_rpc_proc));
  detail::hipcheck(hipMemcpyAsync(d_x, c.h_in.data(), len, hipMemcpyHostToDevice, s), "H2D");
  detail::hipcheck(hipMemcpyAsync(d_off, c.h_off.data(), (n + 1) * 8, hipMemcpyHostToDevice, s), "H2D");
  if (np)
    detail::hipcheck(hipMemcpyAsync(d_p, c.h_off.data() + (n + 1) * 8, np * sizeof(xdrg_rpc_proc),
                                    hipMemcpyHostToDevice, s), "H2D");
  detail::abicheck(xdrg_rpc_dispatch(d_x, len, d_off, n, d_p, std::uint32_t(np), d_h, s), "xdrg_rpc_dispatch");
  c.h_out.resize(n * sizeof(xdrg_rpc_hdr));
  detail::hipcheck(hipMemcpyAsync(c.h_out.data(), d_h, c.h_out.size(), hipMemcpyDeviceToHost, s), "D2H");
  detail::hipcheck(hipStreamSynchronize(s), "sync");
  std::memcpy(h.data(), c.h_out.data(), c.h_out.size());
  for (std::size_t i = 0; i < n; ++i) {
    if (!h[i].err) h[i].body_off -= off[i] + 4;
    h[i].end -= off[i] + 4;
  }
  return h;
}

//! The error reply dispatch sends for each header (rpc_rpc_mismatch_msg,
//! rpc_accepted_error_msg, rpc_prog_mismatch_msg, rpc_auth_error_msg;
//! server.cc:8-67), or nullptr for DISPATCH and dropped messages.
inline std::vector<msg_ptr> rpc_error_replies(const std::vector<xdrg_rpc_hdr> &h,
                                              hipStream_t s = nullptr) {
  context &c = default_context();
  const std::size_t n = h.size();
  std::vector<msg_ptr> out(n);
  if (!n) return out;
  const std::size_t ws_bytes = xdrg_rpc_replies_workspace_size(n);
  xdrg_rpc_hdr *d_h = c.d_nat.get<xdrg_rpc_hdr>(n);
  std::uint8_t *d_out = c.d_xdr.get<std::uint8_t>(36 * n);
  void *ws = c.d_ws.get<std::uint8_t>(ws_bytes);
  std::uint64_t *d_off = c.d_off.get<std::uint64_t>(n + 1);
  c.h_in.resize(n * sizeof(xdrg_rpc_hdr));
  std::memcpy(c.h_in.data(), h.data(), c.h_in.size());
  detail::hipcheck(hipMemcpyAsync(d_h, c.h_in.data(), c.h_in.size(), hipMemcpyHostToDevice, s), "H2D");
  detail::abicheck(xdrg_status_init(c.status(), s), "xdrg_status_init");
  detail::abicheck(xdrg_rpc_replies(d_h, n, d_out, 36 * n, d_off, ws, ws_bytes, c.status(), s), "xdrg_rpc_replies");
  c.h_off.resize((n + 1) * 8);
  c.h_out.resize(36 * n);
  detail::hipcheck(hipMemcpyAsync(c.h_off.data(), d_off, (n + 1) * 8, hipMemcpyDeviceToHost, s), "D2H");
  detail::hipcheck(hipMemcpyAsync(c.h_out.data(), d_out, 36 * n, hipMemcpyDeviceToHost, s), "D2H");
  xdrg_error e{};
  detail::abicheck(xdrg_status_read(c.status(), s, &e), "xdrg_status_read");
  std::vector<std::uint64_t> off(n + 1);
  std::memcpy(off.data(), c.h_off.data(), (n + 1) * 8);
  for (std::size_t i = 0; i < n; ++i) {
    if (off[i + 1] == off[i]) continue;
    out[i] = message_t::alloc(off[i + 1] - off[i] - 4);
    std::memcpy(out[i]->data(), c.h_out.data() + off[i] + 4, out[i]->size());
  }
  return out;
}

}  // namespace gpu
}  // namespace xdr

#endif  // XDRPP_GPU_HH_INCLUDED
