// ORACLE / TEST INFRASTRUCTURE ONLY — never shipped, never measured.
//
// Golden vectors for deeply nested element subroutines, made by the REAL
// reference marshaler (xdrpp/marshal.cc compiled in place) over GENUINE
// xdrc output (oracle/Makefile):
//   test_recursive   tests/xdrtest.x:29-33, chains through `next` of
//                    1 .. 3000 nodes (the lengths straddle the device's
//                    private frames and both deep passes, sub_kernels.h);
//   rp__list         xdrpp/rpcb_prot.x:24-37, the RPCBPROC_DUMP reply
//                    list, 500 entries (plus 33, one past the old bound).
// Chains are written flat (one entry per node) so that no JSON reader
// has to recurse through them:
//   {"test_recursive": [{"nodes": [elem hex, ...], "xdr": hex, "depth": d,
//                        "put_limit": p, "get_limit": g}, ...],
//    "rp__list": [{"nodes": [[prog, vers, netid hex, addr hex, owner hex], ...], ...}]}
// depth: the smallest limit check_xdr_depth accepts; put/get_limit: the
// smallest marshaling_stack_limit under which xdr_to_opaque /
// xdr_from_opaque succeed (both by bisection: they are monotone).
//
//   ref_deep <out.json>
#include <cinttypes>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <xdrpp/depth_checker.h>
#include <xdrpp/marshal.h>

#include "tests/xdrtest.hh"
#include "xdrpp/rpcb_prot.hh"

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

struct rng {  // splitmix64
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint32_t below(uint32_t n) { return n ? uint32_t(next() % n) : 0; }
};
template <typename S> void rbytes(rng &g, S &s, uint32_t maxlen) {
  s.resize(g.below(maxlen + 1));
  for (auto &c : s) c = static_cast<char>(g.below(256));
}

// smallest L in [0, hi] with ok(L) (ok monotone, ok(hi) true)
template <typename F> uint32_t bisect(uint32_t hi, F ok) {
  uint32_t lo = 0;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (ok(mid)) hi = mid; else lo = mid + 1;
  }
  return hi;
}
template <typename F> bool no_overflow(uint32_t L, F f) {
  xdr::marshaling_stack_limit = L;
  bool ok = true;
  try { f(); } catch (const xdr::xdr_stack_overflow &) { ok = false; }
  xdr::marshaling_stack_limit = 0xffffffff;
  return ok;
}

template <typename T> string facts(const T &v, uint32_t nodes) {
  const auto wire = xdr::xdr_to_opaque(v);
  const uint32_t hi = 4 * nodes + 8;
  const uint32_t depth = bisect(hi, [&](uint32_t L) { return xdr::check_xdr_depth(v, L); });
  const uint32_t put = bisect(hi, [&](uint32_t L) { return no_overflow(L, [&] { (void)xdr::xdr_to_opaque(v); }); });
  const uint32_t get = bisect(hi, [&](uint32_t L) {
    return no_overflow(L, [&] { T t; xdr::xdr_from_opaque(wire, t); });
  });
  T back;
  xdr::xdr_from_opaque(wire, back);
  if (!(back == v)) { fprintf(stderr, "round trip mismatch\n"); exit(1); }
  std::ostringstream o;
  o << "\"xdr\": " << q(hex(wire.data(), wire.size())) << ", \"depth\": " << depth
    << ", \"put_limit\": " << put << ", \"get_limit\": " << get;
  return o.str();
}

string chain_record(rng &g, uint32_t nodes) {
  ::test_recursive root;
  std::ostringstream o;
  o << "{\"nodes\": [";
  ::test_recursive *cur = &root;
  for (uint32_t i = 0; i < nodes; ++i) {
    if (i) {
      cur->next.activate();
      cur = cur->next.get();
    }
    rbytes(g, cur->elem, 12);
    o << (i ? ", " : "") << q(hex(cur->elem.data(), cur->elem.size()));
  }
  o << "], " << facts(root, nodes) << "}";
  return o.str();
}

string rpcb_record(rng &g, uint32_t nodes) {
  xdr::rp__list root;
  std::ostringstream o;
  o << "{\"nodes\": [";
  xdr::rp__list *cur = &root;
  for (uint32_t i = 0; i < nodes; ++i) {
    if (i) {
      cur->rpcb_next.activate();
      cur = cur->rpcb_next.get();
    }
    xdr::rpcb &m = cur->rpcb_map;
    m.r_prog = 100000 + g.below(1000);
    m.r_vers = g.below(5);
    rbytes(g, m.r_netid, 8);
    rbytes(g, m.r_addr, 24);
    rbytes(g, m.r_owner, 12);
    o << (i ? ", " : "") << "[" << m.r_prog << ", " << m.r_vers << ", " << q(hex(m.r_netid.data(), m.r_netid.size()))
      << ", " << q(hex(m.r_addr.data(), m.r_addr.size())) << ", " << q(hex(m.r_owner.data(), m.r_owner.size()))
      << "]";
  }
  o << "], " << facts(root, nodes) << "}";
  return o.str();
}

}  // namespace

int main(int argc, char **argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: ref_deep <out.json>\n");
    return 2;
  }
  rng g{0x5EED00D0};
  // main pass: 32 private frames = 33 nodes; deep A: 1024 frames = 1025 nodes
  const uint32_t chains[] = {1, 2, 31, 32, 33, 34, 35, 100, 1000, 1024, 1025, 1026, 1100, 3000};
  std::ofstream f(argv[1]);
  f << "{\"generator\": \"oracle/ref_deep.cc over genuine xdrc output of tests/xdrtest.x and "
       "xdrpp/rpcb_prot.x\",\n\"test_recursive\": [\n";
  for (size_t i = 0; i < sizeof chains / sizeof chains[0]; ++i)
    f << (i ? ",\n" : "") << chain_record(g, chains[i]);
  f << "\n],\n\"rp__list\": [\n" << rpcb_record(g, 33) << ",\n" << rpcb_record(g, 500) << "\n]}\n";
  return f ? 0 : 1;
}
