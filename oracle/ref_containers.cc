// ORACLE / TEST INFRASTRUCTURE ONLY — never shipped, never measured.
//
// Golden vectors for containers of variable-size elements and recursive
// types, made by the REAL reference marshaler (xdrpp/marshal.cc compiled in
// place) over GENUINE xdrc output: tests/xdrtest.hh as the reference's own
// back end (xdrc/gen_hh.cc) emits it from tests/xdrtest.x (oracle/Makefile,
// oracle/xdrc_driver.cc).  Types (tests/xdrtest.x):
//   containertest, containertest1 (:129-137), hasbytes (:94-96),
//   test_recursive (:29-33, depth-bounded), nested_cereal_adapter_calls
//   (:172-176).
//
//   ref_containers <out.json>
//
// For every record: its value (the JSON convention of xdrpp_amd/objects.py:
// bytes as hex, unions as [discriminant, arm], pointers null or the value),
// xdr_to_opaque of it, the smallest depth limit check_xdr_depth accepts,
// and the smallest marshaling_stack_limit under which xdr_to_opaque and
// xdr_from_opaque succeed.  Plus the reference's own error cases: the
// containertest1 overflow of tests/marshal.cc:568-572 and the stack
// overflows just under each record's limits.
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <xdrpp/depth_checker.h>
#include <xdrpp/marshal.h>

#include "tests/xdrtest.hh"
#include "xdrtest_gen.hh"

using namespace testns;
using std::string;
using std::vector;

namespace {

string hex(const void *p, size_t n) {
  static const char *d = "0123456789abcdef";
  string s;
  const uint8_t *b = static_cast<const uint8_t *>(p);
  for (size_t i = 0; i < n; ++i) { s += d[b[i] >> 4]; s += d[b[i] & 15]; }
  return s;
}
string q(const string &s) { return "\"" + s + "\""; }

// ---- JSON writers
template <uint32_t N> string J(const xdr::xstring<N> &s) { return q(hex(s.data(), s.size())); }
template <uint32_t N> string J(const xdr::opaque_vec<N> &s) { return q(hex(s.data(), s.size())); }
template <uint32_t N> string J(const xdr::opaque_array<N> &s) { return q(hex(s.data(), s.size())); }
string J(int32_t v) { return std::to_string(v); }
string J(double v) {
  char b[64];
  snprintf(b, sizeof b, "%.17g", v);
  return b;
}
string J(const fix_4 &f);
string J(const fix_12 &f);
string J(const u_4_12 &u);
string J(const bytes &b);
string J(const test_recursive &t);
template <typename T, uint32_t N> string J(const xdr::xvector<T, N> &v);
template <typename T, uint32_t N> string J(const xdr::xarray<T, N> &v);
template <typename T> string J(const xdr::pointer<T> &p) { return p ? J(*p) : "null"; }
string J(const fix_4 &f) { return "{\"i\": " + J(f.i) + "}"; }
string J(const fix_12 &f) { return "{\"i\": " + J(f.i) + ", \"d\": " + J(f.d) + "}"; }
string J(const u_4_12 &u) {
  return "[" + J(u.which()) + ", " + (u.which() == 4 ? J(u.f4()) : J(u.f12())) + "]";
}
string J(const bytes &b) {
  return "{\"s\": " + J(b.s) + ", \"fixed\": " + J(b.fixed) + ", \"variable\": " + J(b.variable) + "}";
}
string J(const hasbytes &h) { return "{\"the_bytes\": " + J(h.the_bytes) + "}"; }
string J(const test_recursive &t) {
  return "{\"elem\": " + J(t.elem) + ", \"next\": " + J(t.next) + ", \"nextvec\": " + J(t.nextvec) + "}";
}
string J(const containertest &c) { return "{\"uvec\": " + J(c.uvec) + ", \"sarr\": " + J(c.sarr) + "}"; }
string J(const containertest1 &c) { return "{\"uvec\": " + J(c.uvec) + ", \"sarr\": " + J(c.sarr) + "}"; }
string J(const nested_cereal_adapter_calls &c) {
  return "{\"strptr\": " + J(c.strptr) + ", \"strvec\": " + J(c.strvec) + ", \"strarr\": " + J(c.strarr) + "}";
}
template <typename T, uint32_t N> string J(const xdr::xvector<T, N> &v) {
  string s = "[";
  for (size_t i = 0; i < v.size(); ++i) s += (i ? ", " : "") + J(v[i]);
  return s + "]";
}
template <typename T, uint32_t N> string J(const xdr::xarray<T, N> &v) {
  string s = "[";
  for (size_t i = 0; i < N; ++i) s += (i ? ", " : "") + J(v[i]);
  return s + "]";
}

// The smallest marshaling_stack_limit under which f() does not throw
// xdr_stack_overflow.
template <typename F> uint32_t min_limit(F f) {
  for (uint32_t L = 0;; ++L) {
    xdr::marshaling_stack_limit = L;
    try {
      f();
      xdr::marshaling_stack_limit = 0xffffffff;
      return L;
    } catch (const xdr::xdr_stack_overflow &) {
    }
  }
}

template <typename T> string records(const vector<T> &v) {
  std::ostringstream o;
  o << "{\"records\": [\n";
  for (size_t r = 0; r < v.size(); ++r) {
    const auto wire = xdr::xdr_to_opaque(v[r]);
    uint32_t depth = 0;
    while (!xdr::check_xdr_depth(v[r], depth)) ++depth;
    const uint32_t put = min_limit([&] { (void)xdr::xdr_to_opaque(v[r]); });
    const uint32_t get = min_limit([&] { T t; xdr::xdr_from_opaque(wire, t); });
    T back;
    xdr::xdr_from_opaque(wire, back);
    if (!(back == v[r])) { fprintf(stderr, "round trip mismatch\n"); exit(1); }
    o << "  {\"value\": " << J(v[r]) << ", \"xdr\": " << q(hex(wire.data(), wire.size()))
      << ", \"depth\": " << depth << ", \"put_limit\": " << put << ", \"get_limit\": " << get << "}"
      << (r + 1 < v.size() ? ",\n" : "\n");
  }
  o << "]}";
  return o.str();
}

}  // namespace

int main(int argc, char **argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: ref_containers <out.json>\n");
    return 2;
  }
  xdrtest_gen::batches B = xdrtest_gen::make_batches();
  auto &ct = B.ct;
  auto &ct1 = B.ct1;
  auto &hb = B.hb;
  auto &tr = B.tr;
  auto &nc = B.nc;

  // tests/marshal.cc:548-573: containertest with 4 uvec elements read as
  // containertest1 (uvec<2>) throws xdr_overflow
  string kat;
  {
    const auto b = xdr::xdr_to_opaque(ct[1]);
    string what = "(none)";
    try {
      containertest1 c1;
      xdr::xdr_from_opaque(b, c1);
    } catch (const xdr::xdr_overflow &e) {
      what = e.what();
    }
    kat = "{\"type\": \"containertest1\", \"xdr\": " + q(hex(b.data(), b.size())) +
          ", \"exception\": \"xdr_overflow\", \"what\": " + q(what) + "}";
  }
  string stack_what_put, stack_what_get;
  try {
    xdr::marshaling_stack_limit = 1;
    (void)xdr::xdr_to_opaque(tr.back());
  } catch (const xdr::xdr_stack_overflow &e) {
    stack_what_put = e.what();
  }
  try {
    const auto b = (xdr::marshaling_stack_limit = 0xffffffff, xdr::xdr_to_opaque(tr.back()));
    xdr::marshaling_stack_limit = 1;
    test_recursive t;
    xdr::xdr_from_opaque(b, t);
  } catch (const xdr::xdr_stack_overflow &e) {
    stack_what_get = e.what();
  }
  xdr::marshaling_stack_limit = 0xffffffff;

  std::ofstream f(argv[1]);
  f << "{\"generator\": \"oracle/ref_containers.cc over genuine xdrc output of tests/xdrtest.x\",\n"
    << "\"types\": {\n"
    << "\"containertest\": " << records(ct) << ",\n"
    << "\"containertest1\": " << records(ct1) << ",\n"
    << "\"hasbytes\": " << records(hb) << ",\n"
    << "\"test_recursive\": " << records(tr) << ",\n"
    << "\"nested_cereal_adapter_calls\": " << records(nc) << "\n},\n"
    << "\"kat\": [" << kat << "],\n"
    << "\"stack_what\": {\"put\": " << q(stack_what_put) << ", \"get\": " << q(stack_what_get) << "}\n}\n";
  return f ? 0 : 1;
}
