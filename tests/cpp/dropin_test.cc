// C++ drop-in test: the xdr::gpu layer (include/xdrpp_gpu.hh) over the
// reference's own xdr_traits<T> and exceptions.
//
// TEST INFRASTRUCTURE: built by oracle/Makefile against the reference headers
// and xdrpp/marshal.cc (in place, into oracle/_ref/dropin_test), because
// the types it marshals are xdrpp types and the bytes it compares against
// come from the reference marshaler in the same process.
//
//   dropin_test plans <dir>   (CPU)  write the plans recorded from
//                                    xdr_traits<T> (ops/table/stride) per schema
//   dropin_test stage         (CPU)  stage() == the reference-side staged layout,
//                                    unstage(stage(x)) == x, index_records ==
//                                    the reference's record offsets
//   dropin_test gpu [golden]  (GPU)  to_opaque_batch == xdr_put stream,
//                                    from_opaque_batch round trip, and the
//                                    reference's exceptions on bad input;
//                                    to_msg_batch == xdr_to_msg per record,
//                                    from_msg_batch / from_msg_stream back;
//                                    rpc_dispatch_batch / rpc_error_replies
//                                    against the reference's RPC fixtures
// Types with user validate() hooks, in the shape xdrc emits them: load()
// ends with `using xdr::validate; validate(obj);` (xdrc/gen_hh.cc:244-247),
// and the hook is declared before the traits, as tests/validate.cc does for
// fix_4 (tests/validate.cc:7-9,21-26).
#include <xdrpp/types.h>
#include <chrono>
struct vfix {  // tests/xdrtest.x fix_4: struct fix_4 { int i; };
  std::int32_t i;
};
struct vnest {  // struct vnest { string pre<8>; fix_4 inner; string name<16>; };
  xdr::xstring<8> pre;
  vfix inner;
  xdr::xstring<16> name;
};
void validate(const vfix &f);
void validate(const vnest &v);
namespace xdr {
template <>
struct xdr_traits<::vfix> : xdr_struct_base<field_ptr<::vfix, decltype(::vfix::i), &::vfix::i>> {
  template <typename Archive> static void save(Archive &ar, const ::vfix &obj) { archive(ar, obj.i, "i"); }
  template <typename Archive> static void load(Archive &ar, ::vfix &obj) {
    archive(ar, obj.i, "i");
    using xdr::validate;
    validate(obj);
  }
};
template <>
struct xdr_traits<::vnest>
    : xdr_struct_base<field_ptr<::vnest, decltype(::vnest::pre), &::vnest::pre>,
                      field_ptr<::vnest, decltype(::vnest::inner), &::vnest::inner>,
                      field_ptr<::vnest, decltype(::vnest::name), &::vnest::name>> {
  template <typename Archive> static void save(Archive &ar, const ::vnest &obj) {
    archive(ar, obj.pre, "pre");
    archive(ar, obj.inner, "inner");
    archive(ar, obj.name, "name");
  }
  template <typename Archive> static void load(Archive &ar, ::vnest &obj) {
    archive(ar, obj.pre, "pre");
    archive(ar, obj.inner, "inner");
    archive(ar, obj.name, "name");
    using xdr::validate;
    validate(obj);
  }
};
}  // namespace xdr
// tests/validate.cc:21-26
void validate(const vfix &f) {
  if (f.i == 0) throw xdr::xdr_invariant_failed("fix_4::i has value 0");
}
void validate(const vnest &v) {
  if (v.name == "bad") throw xdr::xdr_invariant_failed("vnest::name is bad");
}

#include "ref_objects.hh"
#include "xdrpp_gpu.hh"

#include <xdrpp/depth_checker.h>

#include <cstdio>
#include <fstream>
#include <functional>

using namespace refobj;

// The record types are genuine xdrc output (oracle/ref_types.hh): the
// recorder enumerates their unions' cases from _xdr_case_values()
// (xdrc/gen_hh.cc:410-432) -- no union_cases specializations.

static int failures = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      ++failures;                                      \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);               \
      std::fprintf(stderr, "\n");                      \
    }                                                  \
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

// reference stream: one xdr_put over all records (= xdr_to_opaque of the pack)
template <typename T>
static std::vector<std::uint8_t> ref_stream(const std::vector<T> &v, std::vector<std::uint64_t> &off) {
  std::size_t total = 0;
  off.assign(v.size() + 1, 0);
  for (std::size_t i = 0; i < v.size(); ++i) {
    off[i] = total;
    total += xdr::xdr_size(v[i]);
  }
  off[v.size()] = total;
  std::vector<std::uint8_t> out(total);
  xdr::xdr_put p(out.data(), out.data() + total);
  for (const T &t : v) xdr::archive(p, t);
  return out;
}

template <typename T>
static void check_stage(const char *name, const std::vector<T> &v) {
  const auto &P = xdr::gpu::plan_for<T>();
  xdr::gpu::staged_batch b = xdr::gpu::stage(v.data(), v.size());
  std::vector<std::uint8_t> nat;
  heap_t h;
  stage(v, nat, h);  // the reference-side staged layout (oracle/ref_objects.hh)
  CHECK(nat.size() == b.native.size(), "%s: staged size %zu vs %zu", name, b.native.size(), nat.size());
  CHECK(std::equal(nat.begin(), nat.end(), b.native.begin()), "%s: staged native bytes differ", name);
  CHECK(h.b.size() == b.heap.size() && std::equal(h.b.begin(), h.b.end(), b.heap.begin()),
        "%s: staged heap differs", name);
  std::vector<T> back(v.size());
  xdr::gpu::unstage(b.native.data(), b.heap.data(), v.size(), back.data());
  bool ok = true;
  for (std::size_t i = 0; i < v.size(); ++i) ok = ok && same(v[i], back[i]);
  CHECK(ok, "%s: unstage(stage(x)) != x", name);
  std::vector<std::uint64_t> off;
  std::vector<std::uint8_t> s = ref_stream(v, off);
  CHECK(xdr::gpu::index_records<T>(s.data(), s.size(), v.size()) == off, "%s: index_records differs",
        name);
  std::printf("stage %s: %zu records, stride %u, identity %d ok\n", name, v.size(), P.stride(),
              int(P.identity()));
}

template <typename T>
static void check_gpu(const char *name, const std::vector<T> &v) {
  std::vector<std::uint64_t> off;
  const std::vector<std::uint8_t> want = ref_stream(v, off);
  xdr::opaque_vec<> got = xdr::gpu::to_opaque_batch(v.data(), v.size());
  CHECK(got.size() == want.size() && std::equal(got.begin(), got.end(), want.begin()),
        "%s: to_opaque_batch differs from xdr_put (%zu vs %zu bytes)", name, got.size(), want.size());
  std::vector<T> back(v.size());
  xdr::gpu::from_opaque_batch(want.data(), want.size(), back.data(), back.size());
  bool ok = true;
  for (std::size_t i = 0; i < v.size(); ++i) ok = ok && same(v[i], back[i]);
  CHECK(ok, "%s: from_opaque_batch(xdr_put stream) != records", name);
  // per-record entry point: the batch of one equals xdr_to_opaque(r)
  xdr::opaque_vec<> one = xdr::gpu::to_opaque_batch(&v[1], 1);
  CHECK(one == xdr::xdr_to_opaque(v[1]), "%s: batch of one differs from xdr_to_opaque", name);
  std::printf("gpu %s: %zu records, %zu bytes bit-exact, round trip ok\n", name, v.size(), want.size());
}

// A context in its steady state: once its buffers have grown to a batch
// size, the calls allocate nothing (no hipMalloc, no pinned host memory),
// and an encode sizes its output with one size pass.
template <typename T>
static void check_steady(const char *name, const std::vector<T> &v) {
  std::vector<std::uint64_t> off;
  const std::vector<std::uint8_t> want = ref_stream(v, off);
  xdr::gpu::context c;
  std::vector<T> back(v.size());
  for (int i = 0; i < 2; ++i) {  // the first call grows the buffers
    (void)xdr::gpu::to_opaque_batch(c, v.data(), v.size());
    xdr::gpu::from_opaque_batch(c, want.data(), want.size(), back.data(), back.size());
  }
  const std::size_t a0 = xdr::gpu::context::allocations();
  for (int i = 0; i < 3; ++i) {
    xdr::opaque_vec<> got = xdr::gpu::to_opaque_batch(c, v.data(), v.size());
    CHECK(got.size() == want.size() && std::equal(got.begin(), got.end(), want.begin()),
          "%s: steady to_opaque_batch differs", name);
    xdr::gpu::from_opaque_batch(c, want.data(), want.size(), back.data(), back.size());
  }
  CHECK(xdr::gpu::context::allocations() == a0, "%s: %zu allocations after the steady state", name,
        xdr::gpu::context::allocations() - a0);
  std::printf("steady %s: 3 encode + decode calls, %zu allocations\n", name, xdr::gpu::context::allocations() - a0);
}

// Host-inclusive rates of the C++ drop-in: records in host memory -> staged
// (pinned) -> device encode -> host opaque_vec, and the decode mirror,
// through one context in its steady state; the reference's single-thread
// xdr_put / xdr_get stream over the same records beside it.
template <typename T>
static void bench_one(const char *name, const std::vector<T> &v, int reps) {
  using clk = std::chrono::steady_clock;
  std::vector<std::uint64_t> off;
  const std::vector<std::uint8_t> want = ref_stream(v, off);
  xdr::gpu::context c;
  std::vector<T> back(v.size());
  for (int i = 0; i < 2; ++i) {
    (void)xdr::gpu::to_opaque_batch(c, v.data(), v.size());
    xdr::gpu::from_opaque_batch(c, want.data(), want.size(), back.data(), back.size());
  }
  double te = 1e30, td = 1e30, tr = 1e30, tg = 1e30;
  for (int r = 0; r < reps; ++r) {
    auto t0 = clk::now();
    xdr::opaque_vec<> got = xdr::gpu::to_opaque_batch(c, v.data(), v.size());
    auto t1 = clk::now();
    xdr::gpu::from_opaque_batch(c, want.data(), want.size(), back.data(), back.size());
    auto t2 = clk::now();
    std::vector<std::uint8_t> out(want.size());
    xdr::xdr_put p(out.data(), out.data() + out.size());
    for (const T &t : v) xdr::archive(p, t);
    auto t3 = clk::now();
    std::vector<T> rb(v.size());
    xdr::xdr_get g(out.data(), out.data() + out.size());
    for (T &t : rb) xdr::archive(g, t);
    auto t4 = clk::now();
    te = std::min(te, std::chrono::duration<double>(t1 - t0).count());
    td = std::min(td, std::chrono::duration<double>(t2 - t1).count());
    tr = std::min(tr, std::chrono::duration<double>(t3 - t2).count());
    tg = std::min(tg, std::chrono::duration<double>(t4 - t3).count());
    CHECK(got.size() == want.size() && std::equal(got.begin(), got.end(), want.begin()), "%s: bench bytes", name);
  }
  const double g = double(want.size()) / double(1ull << 30);
  std::printf("{\"schema\": \"%s\", \"records\": %zu, \"xdr_bytes\": %zu, \"to_opaque_batch_gib_s\": %.3f, "
              "\"from_opaque_batch_gib_s\": %.3f, \"encode_decode_gib_s\": %.3f, "
              "\"reference_1thread_put_gib_s\": %.3f, \"reference_1thread_get_gib_s\": %.3f, \"reps\": %d}\n",
              name, v.size(), want.size(), g / te, g / td, 2 * g / (te + td), g / tr, g / tg, reps);
}

// Record-marked messages: to_msg_batch / to_msg_stream against the
// reference's xdr_to_msg per record; from_msg_batch / from_msg_stream back.
template <typename T>
static void check_msgs(const char *name, const std::vector<T> &v) {
  std::vector<std::uint8_t> want;
  std::vector<xdr::msg_ptr> ref;
  for (const T &x : v) {
    ref.push_back(xdr::xdr_to_msg(x));
    want.insert(want.end(), ref.back()->raw_data(), ref.back()->raw_data() + ref.back()->raw_size());
  }
  std::vector<xdr::msg_ptr> got = xdr::gpu::to_msg_batch(v.data(), v.size());
  bool ok = got.size() == ref.size();
  for (std::size_t i = 0; ok && i < ref.size(); ++i)
    ok = got[i]->raw_size() == ref[i]->raw_size() &&
         !memcmp(got[i]->raw_data(), ref[i]->raw_data(), ref[i]->raw_size());
  CHECK(ok, "%s: to_msg_batch differs from xdr_to_msg", name);
  CHECK(xdr::gpu::to_msg_stream(v.data(), v.size()) == want, "%s: to_msg_stream differs", name);
  std::vector<T> back(v.size());
  xdr::gpu::from_msg_batch(ref, back.data());
  std::vector<T> back2 = xdr::gpu::from_msg_stream<T>(want.data(), want.size());
  ok = back2.size() == v.size();
  for (std::size_t i = 0; ok && i < v.size(); ++i) ok = same(v[i], back[i]) && same(v[i], back2[i]);
  CHECK(ok, "%s: from_msg_batch / from_msg_stream != records", name);
  // xdr_from_msg's errors: record 3's message one word short
  if (v.size() > 4) {
    std::vector<xdr::msg_ptr> bad;
    for (std::size_t i = 0; i < 5; ++i) bad.push_back(xdr::xdr_to_msg(v[i]));
    bad[3]->shrink(bad[3]->size() - 4);
    std::vector<T> a(1), b(5);
    std::string rw, gw;
    try { xdr::xdr_from_msg(bad[3], a[0]); } catch (const xdr::xdr_runtime_error &e) { rw = e.what(); }
    try { xdr::gpu::from_msg_batch(bad, b.data()); } catch (const xdr::xdr_runtime_error &e) { gw = e.what(); }
    CHECK(!rw.empty() && rw == gw, "%s: short message: reference \"%s\" vs gpu \"%s\"", name,
          rw.c_str(), gw.c_str());
  }
  std::printf("msgs %s: %zu messages bit-exact, both decodes ok\n", name, v.size());
}

// xdr_size_batch == xdr::xdr_size per record; check_xdr_depth_batch ==
// xdr::check_xdr_depth per record at every limit that matters.
template <typename T>
static void check_sizes_depths(const char *name, const std::vector<T> &v) {
  std::vector<std::uint32_t> sz = xdr::gpu::xdr_size_batch(v.data(), v.size());
  bool ok = sz.size() == v.size();
  for (std::size_t i = 0; ok && i < v.size(); ++i) ok = sz[i] == xdr::xdr_size(v[i]);
  CHECK(ok, "%s: xdr_size_batch differs from xdr_size", name);
  for (std::uint32_t lim = 0; lim <= 7; ++lim) {
    std::vector<bool> d = xdr::gpu::check_xdr_depth_batch(v.data(), v.size(), lim);
    bool okd = d.size() == v.size();
    for (std::size_t i = 0; okd && i < v.size(); ++i) okd = d[i] == xdr::check_xdr_depth(v[i], lim);
    CHECK(okd, "%s: check_xdr_depth_batch differs from check_xdr_depth at limit %u", name, lim);
  }
  std::printf("sizes+depths %s: %zu records match xdr_size / check_xdr_depth\n", name, v.size());
}

static std::vector<std::uint8_t> slurp(const std::string &path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<std::uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

// RPC header batches: rpc_dispatch_batch / rpc_error_replies on msg_ptrs
// against the reference-generated fixtures (tests/golden/rpccall_1024.*).
static void check_rpc(const std::string &gold) {
  const auto stream = slurp(gold + "/rpccall_1024.stream");
  const auto offb = slurp(gold + "/rpccall_1024.msgoffs");
  const auto procb = slurp(gold + "/rpc_procs.bin");
  const auto want = slurp(gold + "/rpccall_1024.hdrs");
  const auto wrep = slurp(gold + "/rpccall_1024.replies");
  CHECK(!stream.empty() && !want.empty(), "rpc fixtures missing under %s", gold.c_str());
  if (stream.empty() || want.empty()) return;
  const auto *off = reinterpret_cast<const std::uint64_t *>(offb.data());
  const std::size_t n = offb.size() / 8 - 1;
  std::vector<xdr::msg_ptr> msgs;
  for (std::size_t i = 0; i < n; ++i) {
    xdr::msg_ptr m = xdr::message_t::alloc(off[i + 1] - off[i] - 4);
    memcpy(m->data(), stream.data() + off[i] + 4, m->size());
    msgs.push_back(std::move(m));
  }
  xdr::gpu::rpc_registry reg;
  const auto *pt = reinterpret_cast<const xdrg_rpc_proc *>(procb.data());
  for (std::size_t i = 0; i < procb.size() / sizeof(xdrg_rpc_proc); ++i)
    reg.add(pt[i].prog, pt[i].vers,
            pt[i].flags & XDRG_RPC_PROC_IFACE_ONLY ? std::vector<std::uint32_t>{}
                                                   : std::vector<std::uint32_t>{pt[i].proc});
  CHECK(reg.table().size() == procb.size() / sizeof(xdrg_rpc_proc), "rpc registry size");
  std::vector<xdrg_rpc_hdr> h = xdr::gpu::rpc_dispatch_batch(msgs, reg);
  const auto *w = reinterpret_cast<const xdrg_rpc_hdr *>(want.data());
  bool ok = true;
  for (std::size_t i = 0; i < n; ++i) {
    xdrg_rpc_hdr g = h[i];
    if (!g.err) g.body_off += off[i] + 4;  // back to stream offsets
    g.end += off[i] + 4;
    ok = ok && !memcmp(&g, &w[i], sizeof g);
  }
  CHECK(ok, "rpc_dispatch_batch differs from the reference's routing");
  std::vector<xdr::msg_ptr> rep = xdr::gpu::rpc_error_replies(h);
  std::vector<std::uint8_t> cat;
  for (const auto &m : rep)
    if (m) cat.insert(cat.end(), m->raw_data(), m->raw_data() + m->raw_size());
  CHECK(cat == wrep, "rpc_error_replies differ from server.cc's replies");
  // a DISPATCH message's arguments decode from data() + body_off
  for (std::size_t i = 0; i < n; ++i)
    if (h[i].action == XDRG_RPC_DISPATCH) {
      CHECK(h[i].body_off <= h[i].end && h[i].end == msgs[i]->size(), "rpc body offsets");
      break;
    }
  std::printf("rpc: %zu headers routed, %zu reply bytes bit-exact\n", n, cat.size());
}

// Run `f`; return the exception's class name and what(), as the reference would.
static std::pair<std::string, std::string> catch_what(const std::function<void()> &f) {
  try {
    f();
  } catch (const xdr::xdr_overflow &e) {
    return {"xdr_overflow", e.what()};
  } catch (const xdr::xdr_stack_overflow &e) {
    return {"xdr_stack_overflow", e.what()};
  } catch (const xdr::xdr_bad_message_size &e) {
    return {"xdr_bad_message_size", e.what()};
  } catch (const xdr::xdr_bad_discriminant &e) {
    return {"xdr_bad_discriminant", e.what()};
  } catch (const xdr::xdr_should_be_zero &e) {
    return {"xdr_should_be_zero", e.what()};
  } catch (const xdr::xdr_invariant_failed &e) {
    return {"xdr_invariant_failed", e.what()};
  }
  return {"none", ""};
}

template <typename T>
static void check_error(const char *label, const std::vector<std::uint8_t> &bytes, std::size_t n) {
  std::vector<T> a(n), b(n);
  auto ref = catch_what([&] {
    // reference: xdr_from_opaque over the concatenation (one archive)
    xdr::xdr_get g(bytes.data(), bytes.data() + bytes.size());
    for (T &t : a) xdr::archive(g, t);
    g.done();
  });
  auto gpu = catch_what([&] { xdr::gpu::from_opaque_batch(bytes.data(), bytes.size(), b.data(), n); });
  CHECK(ref == gpu, "%s: reference %s(\"%s\") vs gpu %s(\"%s\")", label, ref.first.c_str(),
        ref.second.c_str(), gpu.first.c_str(), gpu.second.c_str());
  std::printf("error %s: %s(\"%s\") matches\n", label, ref.first.c_str(), ref.second.c_str());
}

static void gpu_errors() {
  std::vector<xdr::rpc_msg> m;
  gen_rpc(64, WG_SEED_RPC, m);
  std::vector<std::uint64_t> off;
  std::vector<std::uint8_t> s = ref_stream(m, off);
  {  // unknown mtype in record 5
    auto x = s;
    x[off[5] + 7] = 7;
    check_error<xdr::rpc_msg>("rpc bad mtype", x, m.size());
  }
  {  // trailing bytes
    auto x = s;
    x.insert(x.end(), {0, 0, 0, 0});
    check_error<xdr::rpc_msg>("rpc trailing", x, m.size());
  }
  {  // truncated stream
    auto x = s;
    x.resize(x.size() - 8);
    check_error<xdr::rpc_msg>("rpc short", x, m.size());
  }
  std::vector<recvar> r;
  gen_recvar(32, WG_SEED_RECVAR, r);
  std::vector<std::uint8_t> rs = ref_stream(r, off);
  for (std::size_t i = 0; i < r.size(); ++i) {
    if (r[i].blob.size() % 4 == 0) continue;
    auto x = rs;  // nonzero pad byte after record i's blob
    x[off[i] + 16 + r[i].blob.size()] = 0x5a;
    check_error<recvar>("recvar nonzero pad", x, r.size());
    break;
  }
  std::vector<vecrec> vr;
  gen_vecrec(64, WG_SEED_VECREC, vr);
  std::vector<std::uint8_t> vs = ref_stream(vr, off);
  for (std::size_t i = 0; i < vr.size(); ++i) {
    if (vr[i].opt) {  // pointer count 2 in record i
      auto x = vs;
      x[off[i] + 4 + 4 + 4 * vr[i].vals.size() + 3] = 2;
      check_error<vecrec>("vecrec pointer count 2", x, vr.size());
      break;
    }
  }
  {  // xvector count past its bound in record 3
    auto x = vs;
    x[off[3] + 4 + 3] = 17;
    check_error<vecrec>("vecrec xvector overflow", x, vr.size());
  }
  std::vector<rec128> f;
  gen_rec128(16, WG_SEED_REC128, 0, f);
  std::vector<std::uint8_t> fs = ref_stream(f, off);
  fs.pop_back();
  check_error<rec128>("rec128 size not multiple of 4", fs, f.size());
  fs.resize(fs.size() - 3 - 64);
  check_error<rec128>("rec128 short", fs, f.size());
}

// User validate() hooks in batch decode (xdrc/gen_hh.cc:244-247): the
// first failing hook or device error in the reference's load order wins.
static void gpu_validate() {
  CHECK(xdr::gpu::plan_for<vfix>().validates() && xdr::gpu::plan_for<vfix>().identity(),
        "vfix: identity layout with a validate hook");
  CHECK(!xdr::gpu::plan_for<rec128>().validates(), "rec128 has no validate hook");
  std::vector<std::uint64_t> off;
  std::vector<vfix> f(1000);
  for (std::size_t i = 0; i < f.size(); ++i) f[i].i = std::int32_t(i + 1);
  {  // all valid: decodes, hooks pass
    auto x = ref_stream(f, off);
    std::vector<vfix> back(f.size());
    xdr::gpu::from_opaque_batch(x.data(), x.size(), back.data(), back.size());
    CHECK(std::memcmp(back.data(), f.data(), f.size() * sizeof(vfix)) == 0, "vfix round trip");
  }
  f[3].i = 0;
  check_error<vfix>("vfix hook at record 3", ref_stream(f, off), f.size());
  {  // hook at record 3 and the stream ends inside record 500: the hook first
    auto x = ref_stream(f, off);
    x.resize(off[500]);
    check_error<vfix>("vfix hook at 3 before short stream at 500", x, f.size());
  }
  f[3].i = 4;
  f[700].i = 0;
  {  // device error at 500 before the hook at 700
    auto x = ref_stream(f, off);
    x.resize(off[500]);
    check_error<vfix>("vfix short stream at 500 before hook at 700", x, f.size());
  }
  std::vector<vnest> v(300);
  for (std::size_t i = 0; i < v.size(); ++i) {
    v[i].pre = std::string(i % 9, 'p');
    v[i].inner.i = std::int32_t(i + 1);
    v[i].name = std::string(i % 17, 'n');
  }
  {
    auto x = ref_stream(v, off);
    std::vector<vnest> back(v.size());
    xdr::gpu::from_opaque_batch(x.data(), x.size(), back.data(), back.size());
    bool same = true;
    for (std::size_t i = 0; i < v.size(); ++i)
      same = same && back[i].pre == v[i].pre && back[i].inner.i == v[i].inner.i && back[i].name == v[i].name;
    CHECK(same, "vnest round trip");
  }
  v[10].inner.i = 0;
  {  // inner hook at record 10, then name over its bound in record 10: the hook
    auto x = ref_stream(v, off);
    const std::size_t at = off[10] + 4 + ((v[10].pre.size() + 3) & ~std::size_t(3)) + 4;
    x[at + 3] = 17;  // name length 17 > 16
    check_error<vnest>("vnest inner hook before name bound", x, v.size());
  }
  {  // pre over its bound in record 10, before the inner hook: the bound
    auto x = ref_stream(v, off);
    x[off[10] + 3] = 9;
    check_error<vnest>("vnest pre bound before inner hook", x, v.size());
  }
  v[10].inner.i = 11;
  v[20].name = "bad";
  check_error<vnest>("vnest outer hook at 20", ref_stream(v, off), v.size());
  {  // messages: xdr_from_msg per message, the same order
    std::vector<xdr::msg_ptr> msgs;
    for (const vnest &r : v) msgs.push_back(xdr::xdr_to_msg(r));
    std::vector<vnest> a(v.size()), b(v.size());
    auto ref = catch_what([&] {
      for (std::size_t i = 0; i < msgs.size(); ++i) xdr::xdr_from_msg(msgs[i], a[i]);
    });
    auto gpu = catch_what([&] { xdr::gpu::from_msg_batch(msgs, b.data()); });
    CHECK(ref == gpu, "vnest msgs: reference %s(\"%s\") vs gpu %s(\"%s\")", ref.first.c_str(),
          ref.second.c_str(), gpu.first.c_str(), gpu.second.c_str());
    std::printf("error vnest msgs hook at 20: %s(\"%s\") matches\n", ref.first.c_str(), ref.second.c_str());
  }
}

int main(int argc, char **argv) {
  const std::string mode = argc > 1 ? argv[1] : "stage";
  std::vector<testns::numerics> nu;
  std::vector<rec128> rc;
  std::vector<recvar> rv;
  std::vector<xdr::rpc_msg> rp;
  std::vector<vecrec> vr;
  gen_vecrec(1024, WG_SEED_VECREC, vr);
  gen_numerics(1000, WG_SEED_NUMERICS, nu);
  gen_rec128(1024, WG_SEED_REC128, 0, rc);
  gen_recvar(1024, WG_SEED_RECVAR, rv);
  gen_rpc(1024, WG_SEED_RPC, rp);
  if (mode == "plans") {
    const std::string dir = argc > 2 ? argv[2] : ".";
    write_plan<testns::numerics>(dir, "numerics");
    write_plan<testns_v::numerics>(dir, "numerics_validated");
    write_plan<rec128>(dir, "rec128");
    write_plan<recvar>(dir, "recvar");
    write_plan<xdr::rpc_msg>(dir, "rpc");
    write_plan<vecrec>(dir, "vecrec");
  } else if (mode == "stage") {
    check_stage("numerics", nu);
    check_stage("rec128", rc);
    check_stage("recvar", rv);
    check_stage("rpc", rp);
    check_stage("vecrec", vr);
  } else if (mode == "bench") {
    const std::size_t n = argc > 2 ? std::stoull(argv[2]) : (1u << 20);
    std::vector<rec128> brc;
    std::vector<recvar> brv;
    std::vector<xdr::rpc_msg> brp;
    gen_rec128(n, WG_SEED_REC128, 0, brc);
    gen_recvar(n, WG_SEED_RECVAR, brv);
    gen_rpc(n, WG_SEED_RPC, brp);
    bench_one("rec128", brc, 5);
    bench_one("recvar", brv, 5);
    bench_one("rpc", brp, 5);
  } else if (mode == "gpu") {
    check_steady("rec128", rc);
    check_steady("recvar", rv);
    check_steady("rpc", rp);
    check_gpu("numerics", nu);
    check_gpu("rec128", rc);
    check_gpu("recvar", rv);
    check_gpu("rpc", rp);
    check_gpu("vecrec", vr);
    gpu_errors();
    gpu_validate();
    check_msgs("numerics", nu);
    check_msgs("rec128", rc);
    check_msgs("recvar", rv);
    check_msgs("rpc", rp);
    check_msgs("vecrec", vr);
    check_rpc(argc > 2 ? argv[2] : "tests/golden");
    check_sizes_depths("numerics", nu);
    check_sizes_depths("rec128", rc);
    check_sizes_depths("recvar", rv);
    check_sizes_depths("rpc", rp);
    check_sizes_depths("vecrec", vr);
  } else {
    std::fprintf(stderr, "usage: dropin_test plans <dir> | stage | gpu [golden] | bench [records]\n");
    return 2;
  }
  if (failures) std::fprintf(stderr, "%d failure(s)\n", failures);
  return failures ? 1 : 0;
}
