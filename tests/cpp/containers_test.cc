// C++ drop-in test over GENUINE xdrc output: the xdr::gpu layer
// (include/xdrpp_gpu.hh) on tests/xdrtest.x's containers of variable-size
// elements and its recursive type, as the reference's own back end
// (xdrc/gen_hh.cc) generates them (oracle/_ref/gen/inc/tests/xdrtest.hh).
//
// TEST INFRASTRUCTURE: built by oracle/Makefile against the reference
// headers and libxdrgpu.so; run by tests/test_cpp_dropin.py.
//
//   containers_test plans <dir>   recorded plans, one file per type (CPU)
//   containers_test stage         stage/unstage round trip, record index (CPU)
//   containers_test gpu           batch calls against the reference (GPU)
#include "tests/xdrtest.hh"

#include "xdrpp_gpu.hh"
#include "xdrtest_gen.hh"

#include <xdrpp/depth_checker.h>

#include <cstdio>
#include <fstream>
#include <functional>

using namespace testns;

static int failures = 0;
#define CHECK(c, ...)                                             \
  do {                                                            \
    if (!(c)) {                                                   \
      ++failures;                                                 \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);   \
      std::fprintf(stderr, __VA_ARGS__);                          \
      std::fprintf(stderr, "\n");                                 \
    }                                                             \
  } while (0)

template <typename T> static void write_plan(const std::string &dir, const char *name) {
  const auto &P = xdr::gpu::plan_for<T>();
  std::ofstream f(dir + "/" + name + ".plan", std::ios::binary);
  const std::uint32_t hdr[4] = {static_cast<std::uint32_t>(P.ops().size()),
                                static_cast<std::uint32_t>(P.table().size()), P.stride(),
                                P.identity() ? 1u : 0u};
  f.write(reinterpret_cast<const char *>(hdr), sizeof hdr);
  f.write(reinterpret_cast<const char *>(P.ops().data()), P.ops().size() * sizeof(xdrg_op));
  f.write(reinterpret_cast<const char *>(P.table().data()), P.table().size() * 4);
}

template <typename T>
static std::vector<std::uint8_t> ref_stream(const std::vector<T> &v, std::vector<std::uint64_t> &off) {
  std::vector<std::uint8_t> out;
  off.assign(1, 0);
  for (const T &t : v) {
    const auto b = xdr::xdr_to_opaque(t);
    out.insert(out.end(), b.begin(), b.end());
    off.push_back(out.size());
  }
  return out;
}

template <typename T> static void check_stage(const char *name, const std::vector<T> &v) {
  xdr::gpu::staged_batch b = xdr::gpu::stage(v.data(), v.size());
  std::vector<T> back(v.size());
  xdr::gpu::unstage(b.native.data(), b.heap.data(), v.size(), back.data());
  CHECK(back == v, "%s: unstage(stage(x)) != x", name);
  std::vector<std::uint64_t> off;
  const std::vector<std::uint8_t> s = ref_stream(v, off);
  CHECK(xdr::gpu::index_records<T>(s.data(), s.size(), v.size()) == off, "%s: index_records differs", name);
  std::printf("stage %s: %zu records, %zu heap bytes ok\n", name, v.size(), b.heap.size());
}

template <typename T> static void check_gpu(const char *name, const std::vector<T> &v) {
  std::vector<std::uint64_t> off;
  const std::vector<std::uint8_t> want = ref_stream(v, off);
  xdr::opaque_vec<> got = xdr::gpu::to_opaque_batch(v.data(), v.size());
  CHECK(got.size() == want.size() && std::equal(got.begin(), got.end(), want.begin()),
        "%s: to_opaque_batch differs from xdr_to_opaque (%zu vs %zu bytes)", name, got.size(), want.size());
  std::vector<T> back(v.size());
  xdr::gpu::from_opaque_batch(want.data(), want.size(), back.data(), back.size());
  CHECK(back == v, "%s: from_opaque_batch != records", name);
  const std::vector<std::uint32_t> sz = xdr::gpu::xdr_size_batch(v.data(), v.size());
  bool ok = true;
  for (std::size_t i = 0; i < v.size(); ++i) ok = ok && sz[i] == xdr::xdr_size(v[i]);
  CHECK(ok, "%s: xdr_size_batch differs", name);
  for (std::uint32_t lim = 0; lim <= 14; lim += 2) {
    const std::vector<bool> d = xdr::gpu::check_xdr_depth_batch(v.data(), v.size(), lim);
    bool okd = true;
    for (std::size_t i = 0; i < v.size(); ++i) okd = okd && d[i] == xdr::check_xdr_depth(v[i], lim);
    CHECK(okd, "%s: check_xdr_depth_batch differs at limit %u", name, lim);
  }
  // marshaling_stack_limit: the reference's and the batch's exceptions agree
  for (std::uint32_t lim = 1; lim <= 6; ++lim) {
    xdr::marshaling_stack_limit = lim;
    std::string rw, gw;
    try {
      for (const T &t : v) (void)xdr::xdr_to_opaque(t);
    } catch (const xdr::xdr_runtime_error &e) { rw = e.what(); }
    try {
      (void)xdr::gpu::to_opaque_batch(v.data(), v.size());
    } catch (const xdr::xdr_runtime_error &e) { gw = e.what(); }
    xdr::marshaling_stack_limit = 0xffffffff;
    CHECK(rw == gw, "%s: stack limit %u: reference \"%s\" vs gpu \"%s\"", name, lim, rw.c_str(), gw.c_str());
  }
  std::printf("gpu %s: %zu records, %zu bytes bit-exact, round trip, sizes, depths, limits ok\n", name,
              v.size(), want.size());
}

static std::string catch_what(const std::function<void()> &f) {
  try {
    f();
  } catch (const xdr::xdr_runtime_error &e) {
    return e.what();
  }
  return "";
}

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: containers_test plans <dir> | stage | gpu\n");
    return 2;
  }
  const std::string mode = argv[1];
  if (mode == "plans" && argc == 3) {
    write_plan<containertest>(argv[2], "containertest");
    write_plan<containertest1>(argv[2], "containertest1");
    write_plan<hasbytes>(argv[2], "hasbytes");
    write_plan<test_recursive>(argv[2], "test_recursive");
    write_plan<nested_cereal_adapter_calls>(argv[2], "nested_cereal_adapter_calls");
    return 0;
  }
  const xdrtest_gen::batches B = xdrtest_gen::make_batches();
  if (mode == "stage") {
    check_stage("containertest", B.ct);
    check_stage("containertest1", B.ct1);
    check_stage("hasbytes", B.hb);
    check_stage("test_recursive", B.tr);
    check_stage("nested_cereal_adapter_calls", B.nc);
  } else if (mode == "gpu") {
    check_gpu("containertest", B.ct);
    check_gpu("containertest1", B.ct1);
    check_gpu("hasbytes", B.hb);
    check_gpu("test_recursive", B.tr);
    check_gpu("nested_cereal_adapter_calls", B.nc);
    // tests/marshal.cc:568-572: containertest's 4 uvec elements read as
    // containertest1 (uvec<2>) -> xdr_overflow, batch and reference alike
    const auto b = xdr::xdr_to_opaque(B.ct[1]);
    const std::string rw = catch_what([&] { containertest1 c; xdr::xdr_from_opaque(b, c); });
    const std::string gw = catch_what([&] {
      containertest1 c;
      xdr::gpu::from_opaque_batch(b.data(), b.size(), &c, 1);
    });
    CHECK(!rw.empty() && rw == gw, "containertest1: reference \"%s\" vs gpu \"%s\"", rw.c_str(), gw.c_str());
    std::printf("containertest1 overflow: \"%s\" ok\n", gw.c_str());
  } else {
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  if (failures) std::fprintf(stderr, "%d failure(s)\n", failures);
  return failures ? 1 : 0;
}
