// -*- C++ -*-
// ORACLE / TEST INFRASTRUCTURE ONLY.  Never linked into the product.
//
// The four benchmark schemas expressed as xdrpp types with xdr_traits
// specializations written exactly in the form xdrc's back end emits them:
//   structs:  xdr_struct_base<field_ptr<...>...> + save/load calling
//             archive(ar, obj.f, "f") in declaration order, load ending in
//             validate(obj)                      (xdrc/gen_hh.cc:212-250)
//   enums:    xdr_integral_base<E, uint32_t> + is_enum + enum_name/values
//                                                (xdrc/gen_hh.cc:271-305)
//   unions:   discriminant first, then the selected arm; unknown
//             discriminant -> xdr_bad_discriminant("bad value of <tag> in
//             <union>")                          (xdrc/gen_hh.cc:639-673)
// The xdrc front end (flex/bison) is not available in this image, so the
// schemas are hand-expanded; they are compiled against the reference
// headers in place (-I /root/reference), never copied.
//
// numerics follows tests/xdrtest.x:98-107; rpc types follow
// xdrpp/rpc_msg.x:5-140; rec128 / recvar are the north-star schemas of
// SURVEY.md §8.
#pragma once
#include <xdrpp/marshal.h>

#define XF(T, f) xdr::field_ptr<T, decltype(T::f), &T::f>

// ---------------------------------------------------------------- numerics
namespace testns {
enum other_color : std::int32_t { RED, REDDER, REDDEST };
struct numerics {
  bool b;
  std::int32_t i1;
  std::uint32_t i2;
  std::int64_t i3;
  std::uint64_t i4;
  float f1;
  double f2;
  other_color e1;
};
}  // namespace testns

// Same struct in a namespace that opts in to enum validation
// (tests/validate.cc:18-20 idiom).
namespace testns_v {
enum other_color : std::int32_t { RED, REDDER, REDDEST };
template <typename T> inline void xdr_validate_enum(T);
struct numerics {
  bool b;
  std::int32_t i1;
  std::uint32_t i2;
  std::int64_t i3;
  std::uint64_t i4;
  float f1;
  double f2;
  other_color e1;
};
}  // namespace testns_v

namespace xdr {
#define ENUM_TRAITS(E)                                                    \
  template <> struct xdr_traits<E::other_color>                          \
      : xdr_integral_base<E::other_color, std::uint32_t> {               \
    using case_type = std::int32_t;                                       \
    static Constexpr const bool is_enum = true;                           \
    static Constexpr const bool is_numeric = false;                       \
    static const char *enum_name(E::other_color val) {                   \
      switch (val) {                                                      \
      case E::RED: return "RED";                                          \
      case E::REDDER: return "REDDER";                                    \
      case E::REDDEST: return "REDDEST";                                  \
      default: return nullptr;                                            \
      }                                                                   \
    }                                                                     \
    static const std::vector<int32_t> &enum_values() {                    \
      static const std::vector<int32_t> v = {E::RED, E::REDDER, E::REDDEST}; \
      return v;                                                           \
    }                                                                     \
  };
ENUM_TRAITS(testns)
ENUM_TRAITS(testns_v)

#define NUMERICS_TRAITS(NS)                                               \
  template <>                                                             \
  struct xdr_traits<NS::numerics>                                         \
      : xdr_struct_base<XF(NS::numerics, b), XF(NS::numerics, i1),        \
                        XF(NS::numerics, i2), XF(NS::numerics, i3),       \
                        XF(NS::numerics, i4), XF(NS::numerics, f1),       \
                        XF(NS::numerics, f2), XF(NS::numerics, e1)> {     \
    template <typename Archive>                                           \
    static void save(Archive &ar, const NS::numerics &obj) {              \
      archive(ar, obj.b, "b"); archive(ar, obj.i1, "i1");                 \
      archive(ar, obj.i2, "i2"); archive(ar, obj.i3, "i3");               \
      archive(ar, obj.i4, "i4"); archive(ar, obj.f1, "f1");               \
      archive(ar, obj.f2, "f2"); archive(ar, obj.e1, "e1");               \
    }                                                                     \
    template <typename Archive>                                           \
    static void load(Archive &ar, NS::numerics &obj) {                    \
      archive(ar, obj.b, "b"); archive(ar, obj.i1, "i1");                 \
      archive(ar, obj.i2, "i2"); archive(ar, obj.i3, "i3");               \
      archive(ar, obj.i4, "i4"); archive(ar, obj.f1, "f1");               \
      archive(ar, obj.f2, "f2"); archive(ar, obj.e1, "e1");               \
      using xdr::validate;                                                \
      validate(obj);                                                      \
    }                                                                     \
  };
NUMERICS_TRAITS(testns)
NUMERICS_TRAITS(testns_v)
}  // namespace xdr

// ------------------------------------------------------------------ rec128
// struct rec128 { int a0..a7; unsigned hyper u0..u5; double d0..d5; };
struct rec128 {
  std::int32_t a0, a1, a2, a3, a4, a5, a6, a7;
  std::uint64_t u0, u1, u2, u3, u4, u5;
  double d0, d1, d2, d3, d4, d5;
};
static_assert(sizeof(rec128) == 128, "rec128 native layout");

namespace xdr {
template <>
struct xdr_traits<::rec128>
    : xdr_struct_base<XF(::rec128, a0), XF(::rec128, a1), XF(::rec128, a2),
                      XF(::rec128, a3), XF(::rec128, a4), XF(::rec128, a5),
                      XF(::rec128, a6), XF(::rec128, a7), XF(::rec128, u0),
                      XF(::rec128, u1), XF(::rec128, u2), XF(::rec128, u3),
                      XF(::rec128, u4), XF(::rec128, u5), XF(::rec128, d0),
                      XF(::rec128, d1), XF(::rec128, d2), XF(::rec128, d3),
                      XF(::rec128, d4), XF(::rec128, d5)> {
#define REC128_FIELDS(X)                                                    \
  X(a0) X(a1) X(a2) X(a3) X(a4) X(a5) X(a6) X(a7) X(u0) X(u1) X(u2) X(u3)   \
  X(u4) X(u5) X(d0) X(d1) X(d2) X(d3) X(d4) X(d5)
#define ARCH(f) archive(ar, obj.f, #f);
  template <typename Archive> static void save(Archive &ar, const ::rec128 &obj) {
    REC128_FIELDS(ARCH)
  }
  template <typename Archive> static void load(Archive &ar, ::rec128 &obj) {
    REC128_FIELDS(ARCH)
    using xdr::validate;
    validate(obj);
  }
#undef ARCH
};
}  // namespace xdr

// ------------------------------------------------------------------ recvar
// struct recvar { unsigned hyper id; int kind; opaque blob<256>;
//                 string name<64>; double score; };
struct recvar {
  std::uint64_t id;
  std::int32_t kind;
  xdr::opaque_vec<256> blob;
  xdr::xstring<64> name;
  double score;
};
namespace xdr {
template <>
struct xdr_traits<::recvar>
    : xdr_struct_base<XF(::recvar, id), XF(::recvar, kind), XF(::recvar, blob),
                      XF(::recvar, name), XF(::recvar, score)> {
#define RECVAR_FIELDS(X) X(id) X(kind) X(blob) X(name) X(score)
#define ARCH(f) archive(ar, obj.f, #f);
  template <typename Archive> static void save(Archive &ar, const ::recvar &obj) {
    RECVAR_FIELDS(ARCH)
  }
  template <typename Archive> static void load(Archive &ar, ::recvar &obj) {
    RECVAR_FIELDS(ARCH)
    using xdr::validate;
    validate(obj);
  }
#undef ARCH
};
}  // namespace xdr

// --------------------------------------------------------- rpc_msg (RFC 5531)
// Mirrors xdrpp/rpc_msg.x:5-140.  Unions keep every arm as a member (only
// the selected one is marshaled), which is byte-for-byte what xdrc's
// union classes marshal.  Enum-typed fields are carried as their int32
// representation (enums are int32 bit patterns on the wire and, without
// xdr_validate_enum, are not range-checked).
namespace rpcx {
enum : std::int32_t { AUTH_NONE = 0, AUTH_SYS = 1 };
enum : std::int32_t { CALL = 0, REPLY = 1 };
enum : std::int32_t { MSG_ACCEPTED = 0, MSG_DENIED = 1 };
enum : std::int32_t { SUCCESS = 0, PROG_UNAVAIL = 1, PROG_MISMATCH = 2 };
enum : std::int32_t { RPC_MISMATCH = 0, AUTH_ERROR = 1 };

struct opaque_auth {
  std::int32_t flavor;
  xdr::opaque_vec<400> body;
};
struct mismatch_info {
  std::uint32_t low;
  std::uint32_t high;
};
struct call_body {
  std::uint32_t rpcvers, prog, vers, proc;
  opaque_auth cred;
  opaque_auth verf;
};
// accepted_reply::reply_data (xdrc names the anonymous union _reply_data_t)
struct reply_data_u {
  std::int32_t stat = SUCCESS;
  xdr::opaque_array<0> results;
  mismatch_info mismatch_info_{};
};
struct accepted_reply {
  opaque_auth verf;
  reply_data_u reply_data;
};
struct rejected_reply {
  std::int32_t stat = RPC_MISMATCH;
  mismatch_info mismatch_info_{};
  std::int32_t rj_why = 0;
};
struct reply_body {
  std::int32_t stat = MSG_ACCEPTED;
  accepted_reply areply;
  rejected_reply rreply;
};
// rpc_msg::body (xdrc: _body_t)
struct body_u {
  std::int32_t mtype = CALL;
  call_body cbody;
  reply_body rbody;
};
struct rpc_msg {
  std::uint32_t xid;
  body_u body;
};
}  // namespace rpcx

namespace xdr {
#define RPC_STRUCT2(T, f1, f2)                                               \
  template <> struct xdr_traits<T> : xdr_struct_base<XF(T, f1), XF(T, f2)> { \
    template <typename A> static void save(A &ar, const T &obj) {           \
      archive(ar, obj.f1, #f1); archive(ar, obj.f2, #f2);                    \
    }                                                                        \
    template <typename A> static void load(A &ar, T &obj) {                 \
      archive(ar, obj.f1, #f1); archive(ar, obj.f2, #f2);                    \
      using xdr::validate; validate(obj);                                    \
    }                                                                        \
  };
RPC_STRUCT2(rpcx::opaque_auth, flavor, body)
RPC_STRUCT2(rpcx::mismatch_info, low, high)

template <>
struct xdr_traits<rpcx::call_body>
    : xdr_struct_base<XF(rpcx::call_body, rpcvers), XF(rpcx::call_body, prog),
                      XF(rpcx::call_body, vers), XF(rpcx::call_body, proc),
                      XF(rpcx::call_body, cred), XF(rpcx::call_body, verf)> {
  template <typename A> static void save(A &ar, const rpcx::call_body &obj) {
    archive(ar, obj.rpcvers, "rpcvers"); archive(ar, obj.prog, "prog");
    archive(ar, obj.vers, "vers"); archive(ar, obj.proc, "proc");
    archive(ar, obj.cred, "cred"); archive(ar, obj.verf, "verf");
  }
  template <typename A> static void load(A &ar, rpcx::call_body &obj) {
    archive(ar, obj.rpcvers, "rpcvers"); archive(ar, obj.prog, "prog");
    archive(ar, obj.vers, "vers"); archive(ar, obj.proc, "proc");
    archive(ar, obj.cred, "cred"); archive(ar, obj.verf, "verf");
    using xdr::validate; validate(obj);
  }
};

// Union traits in the shape of gen_hh.cc:575-675: serial_size/save throw on
// an unknown discriminant; load reads the discriminant, validates it (the
// generated tag setter, gen_hh.cc:472-487) and then reads the arm.
#define RPC_UNION_BEGIN(T)                                                 \
  template <> struct xdr_traits<T> : xdr_traits_base {                     \
    static Constexpr const bool is_class = true;                           \
    static Constexpr const bool is_union = true;                           \
    static Constexpr const bool has_fixed_size = false;

RPC_UNION_BEGIN(rpcx::reply_data_u)
  static void bad() { throw xdr_bad_discriminant("bad value of stat in _reply_data_t"); }
  static std::size_t serial_size(const rpcx::reply_data_u &o) {
    switch (o.stat) {
    case rpcx::SUCCESS: return 4 + xdr_size(o.results);
    case rpcx::PROG_MISMATCH: return 4 + xdr_size(o.mismatch_info_);
    default: return 4;
    }
  }
  template <typename A> static void save(A &ar, const rpcx::reply_data_u &o) {
    archive(ar, o.stat, "stat");
    switch (o.stat) {
    case rpcx::SUCCESS: archive(ar, o.results, "results"); break;
    case rpcx::PROG_MISMATCH: archive(ar, o.mismatch_info_, "mismatch_info"); break;
    default: break;
    }
  }
  template <typename A> static void load(A &ar, rpcx::reply_data_u &o) {
    std::int32_t which;
    archive(ar, which, "stat");
    o.stat = which;
    switch (o.stat) {
    case rpcx::SUCCESS: archive(ar, o.results, "results"); break;
    case rpcx::PROG_MISMATCH: archive(ar, o.mismatch_info_, "mismatch_info"); break;
    default: break;
    }
  }
};

RPC_STRUCT2(rpcx::accepted_reply, verf, reply_data)

RPC_UNION_BEGIN(rpcx::rejected_reply)
  static void bad() { throw xdr_bad_discriminant("bad value of stat in rejected_reply"); }
  static std::size_t serial_size(const rpcx::rejected_reply &o) {
    switch (o.stat) {
    case rpcx::RPC_MISMATCH: return 4 + xdr_size(o.mismatch_info_);
    case rpcx::AUTH_ERROR: return 8;
    default: bad(); return 0;
    }
  }
  template <typename A> static void save(A &ar, const rpcx::rejected_reply &o) {
    archive(ar, o.stat, "stat");
    switch (o.stat) {
    case rpcx::RPC_MISMATCH: archive(ar, o.mismatch_info_, "mismatch_info"); break;
    case rpcx::AUTH_ERROR: archive(ar, o.rj_why, "rj_why"); break;
    default: bad();
    }
  }
  template <typename A> static void load(A &ar, rpcx::rejected_reply &o) {
    std::int32_t which;
    archive(ar, which, "stat");
    if (which != rpcx::RPC_MISMATCH && which != rpcx::AUTH_ERROR) bad();
    o.stat = which;
    if (o.stat == rpcx::RPC_MISMATCH)
      archive(ar, o.mismatch_info_, "mismatch_info");
    else
      archive(ar, o.rj_why, "rj_why");
  }
};

RPC_UNION_BEGIN(rpcx::reply_body)
  static void bad() { throw xdr_bad_discriminant("bad value of stat in reply_body"); }
  static std::size_t serial_size(const rpcx::reply_body &o) {
    switch (o.stat) {
    case rpcx::MSG_ACCEPTED: return 4 + xdr_size(o.areply);
    case rpcx::MSG_DENIED: return 4 + xdr_size(o.rreply);
    default: bad(); return 0;
    }
  }
  template <typename A> static void save(A &ar, const rpcx::reply_body &o) {
    archive(ar, o.stat, "stat");
    switch (o.stat) {
    case rpcx::MSG_ACCEPTED: archive(ar, o.areply, "areply"); break;
    case rpcx::MSG_DENIED: archive(ar, o.rreply, "rreply"); break;
    default: bad();
    }
  }
  template <typename A> static void load(A &ar, rpcx::reply_body &o) {
    std::int32_t which;
    archive(ar, which, "stat");
    if (which != rpcx::MSG_ACCEPTED && which != rpcx::MSG_DENIED) bad();
    o.stat = which;
    if (o.stat == rpcx::MSG_ACCEPTED)
      archive(ar, o.areply, "areply");
    else
      archive(ar, o.rreply, "rreply");
  }
};

RPC_UNION_BEGIN(rpcx::body_u)
  static void bad() { throw xdr_bad_discriminant("bad value of mtype in _body_t"); }
  static std::size_t serial_size(const rpcx::body_u &o) {
    switch (o.mtype) {
    case rpcx::CALL: return 4 + xdr_size(o.cbody);
    case rpcx::REPLY: return 4 + xdr_size(o.rbody);
    default: bad(); return 0;
    }
  }
  template <typename A> static void save(A &ar, const rpcx::body_u &o) {
    archive(ar, o.mtype, "mtype");
    switch (o.mtype) {
    case rpcx::CALL: archive(ar, o.cbody, "cbody"); break;
    case rpcx::REPLY: archive(ar, o.rbody, "rbody"); break;
    default: bad();
    }
  }
  template <typename A> static void load(A &ar, rpcx::body_u &o) {
    std::int32_t which;
    archive(ar, which, "mtype");
    if (which != rpcx::CALL && which != rpcx::REPLY) bad();
    o.mtype = which;
    if (o.mtype == rpcx::CALL)
      archive(ar, o.cbody, "cbody");
    else
      archive(ar, o.rbody, "rbody");
  }
};
RPC_STRUCT2(rpcx::rpc_msg, xid, body)
}  // namespace xdr

// ------------------------------------------------------------------ vecrec
// Counted and optional containers of fixed-size elements:
//   struct vpair { hyper h; bool b; };
//   struct vecrec { unsigned id; int vals<16>; mismatch_info *opt;
//                   vpair pairs<8>; bool flag; };
struct vpair {
  std::int64_t h;
  bool b;
};
struct vecrec {
  std::uint32_t id;
  xdr::xvector<std::int32_t, 16> vals;
  xdr::pointer<rpcx::mismatch_info> opt;
  xdr::xvector<vpair, 8> pairs;
  bool flag;
};
namespace xdr {
template <>
struct xdr_traits<::vpair> : xdr_struct_base<XF(::vpair, h), XF(::vpair, b)> {
  template <typename A> static void save(A &ar, const ::vpair &obj) {
    archive(ar, obj.h, "h"); archive(ar, obj.b, "b");
  }
  template <typename A> static void load(A &ar, ::vpair &obj) {
    archive(ar, obj.h, "h"); archive(ar, obj.b, "b");
    using xdr::validate; validate(obj);
  }
};
template <>
struct xdr_traits<::vecrec>
    : xdr_struct_base<XF(::vecrec, id), XF(::vecrec, vals), XF(::vecrec, opt),
                      XF(::vecrec, pairs), XF(::vecrec, flag)> {
#define VECREC_FIELDS(X) X(id) X(vals) X(opt) X(pairs) X(flag)
#define ARCH(f) archive(ar, obj.f, #f);
  template <typename Archive> static void save(Archive &ar, const ::vecrec &obj) {
    VECREC_FIELDS(ARCH)
  }
  template <typename Archive> static void load(Archive &ar, ::vecrec &obj) {
    VECREC_FIELDS(ARCH)
    using xdr::validate;
    validate(obj);
  }
#undef ARCH
};
}  // namespace xdr
