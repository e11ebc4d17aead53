// ORACLE / TEST INFRASTRUCTURE ONLY.
//
// Seeded values of tests/xdrtest.x's container types over the GENUINE
// xdrc-generated tests/xdrtest.hh, shared by oracle/ref_containers.cc (the
// reference fixtures) and tests/cpp/containers_test.cc (the C++ layer).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace xdrtest_gen {
using namespace testns;
using std::vector;

struct rng {  // splitmix64
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint32_t below(uint32_t n) { return n ? uint32_t(next() % n) : 0; }
  bool coin() { return next() & 1; }
};

template <typename S> void rbytes(rng &g, S &s, uint32_t maxlen) {
  s.resize(g.below(maxlen + 1));
  for (auto &c : s) c = static_cast<char>(g.below(256));
}
inline u_4_12 ru(rng &g) {
  u_4_12 u(g.coin() ? 4 : 12);
  if (u.which() == 4) u.f4().i = int32_t(g.next());
  else { u.f12().i = int32_t(g.next()); u.f12().d = double(int32_t(g.next())) / 8.0; }
  return u;
}
inline containertest r_containertest(rng &g) {
  containertest c;
  c.uvec.resize(g.below(7));
  for (auto &u : c.uvec) u = ru(g);
  for (auto &s : c.sarr) rbytes(g, s, 40);
  return c;
}
inline containertest1 r_containertest1(rng &g) {
  containertest1 c;
  c.uvec.resize(g.below(3));
  for (auto &u : c.uvec) u = ru(g);
  for (auto &s : c.sarr) rbytes(g, s, 40);
  return c;
}
inline hasbytes r_hasbytes(rng &g) {
  hasbytes h;
  h.the_bytes.resize(g.below(6));
  for (auto &b : h.the_bytes) {
    rbytes(g, b.s, 16);
    for (auto &c : b.fixed) c = uint8_t(g.below(256));
    rbytes(g, b.variable, 16);
  }
  return h;
}
inline test_recursive r_recursive(rng &g, int depth) {
  test_recursive t;
  rbytes(g, t.elem, 12);
  if (depth > 0 && g.coin()) t.next.activate() = r_recursive(g, depth - 1);
  if (depth > 0) {
    t.nextvec.resize(g.below(4));
    for (auto &e : t.nextvec) e = r_recursive(g, depth - 1);
  }
  return t;
}
inline nested_cereal_adapter_calls r_nested(rng &g) {
  nested_cereal_adapter_calls c;
  if (g.coin()) rbytes(g, c.strptr.activate(), 32);
  c.strvec.resize(g.below(6));
  for (auto &s : c.strvec) rbytes(g, s, 32);
  for (auto &s : c.strarr) rbytes(g, s, 32);
  return c;
}

// The batches of tests/golden/containers.json, in its order.
struct batches {
  vector<containertest> ct;
  vector<containertest1> ct1;
  vector<hasbytes> hb;
  vector<test_recursive> tr;
  vector<nested_cereal_adapter_calls> nc;
};
inline batches make_batches() {
  batches B;
  auto &ct = B.ct;
  auto &ct1 = B.ct1;
  auto &hb = B.hb;
  auto &tr = B.tr;
  auto &nc = B.nc;
  rng g{0x5EED0A8ull};
  // edge cases first: every container empty, then the reference's own value
  ct.emplace_back();
  {
    containertest c;  // tests/marshal.cc:551-553
    c.uvec = {u_4_12(4), u_4_12(12), u_4_12(4), u_4_12(4)};
    c.sarr[0] = "hello";
    c.sarr[1] = "world";
    ct.push_back(c);
  }
  ct1.emplace_back();
  hb.emplace_back();
  tr.emplace_back();
  nc.emplace_back();
  for (int i = 0; i < 200; ++i) {
    ct.push_back(r_containertest(g));
    ct1.push_back(r_containertest1(g));
    hb.push_back(r_hasbytes(g));
    tr.push_back(r_recursive(g, 1 + int(g.below(5))));
    nc.push_back(r_nested(g));
  }
  {
    test_recursive deep;  // a chain 12 deep through `next`
    test_recursive *t = &deep;
    for (int d = 0; d < 12; ++d) { t->elem = "n" + std::to_string(d); t = &t->next.activate(); }
    tr.push_back(deep);
  }

  return B;
}

}  // namespace xdrtest_gen
