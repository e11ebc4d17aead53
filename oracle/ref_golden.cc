// ORACLE / TEST INFRASTRUCTURE ONLY — never shipped, never measured as
// the product.
//
// Drives the REAL reference marshaler (xdrpp/marshal.{h,cc}, compiled from
// /root/reference in place by oracle/Makefile) over the four benchmark
// workloads and writes golden fixtures, plus a CPU timing mode used as the
// "reference" CPU baseline.
//
//   ref_golden gen   <schema> <n> <outprefix>
//       writes <outprefix>.native (staged native records), .heap (var
//       payload heap), .xdr (concatenated xdr_put output) and .offsets
//       (n+1 little-endian u64 record offsets).  The XDR bytes are produced
//       by one xdr_put archive over the whole buffer (= xdr_to_opaque of the
//       argument pack, xdrpp/marshal.h:264-272); each record is also
//       checked against its own xdr_to_opaque and round-tripped through
//       xdr_from_opaque (marshal.h:299-306).
//   ref_golden kat   <outfile.json>
//       known-answer vectors and error cases (exception class + what()).
//   ref_golden bench <schema> <n> <threads> <reps>
//       times xdr_put / xdr_get streams over contiguous slices, one
//       std::thread per slice, and per-record xdr_to_opaque; prints JSON.
#include "ref_objects.hh"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

using std::size_t;
using std::string;
using std::vector;

using namespace refobj;

template <typename T>
static void emit(const vector<T> &v, const string &prefix, bool with_msgs = true) {
  vector<uint8_t> nat;
  heap_t heap;
  stage(v, nat, heap);
  vector<uint64_t> off(v.size() + 1, 0);
  for (size_t r = 0; r < v.size(); ++r) off[r + 1] = off[r] + xdr::xdr_size(v[r]);
  vector<uint8_t> out(off.back());
  {
    // One archive over the whole stream: xdr_to_opaque(r0, ..., rn-1).
    xdr::xdr_put p(out.data(), out.data() + out.size());
    for (const T &x : v) archive(p, x);
    if (p.p_ != p.e_) die("size mismatch");
  }
  // Spot-check per-record xdr_to_opaque and the round trip (all records
  // for small n, a stride sample for large n).
  size_t step = v.size() <= 65536 ? 1 : v.size() / 4096;
  for (size_t r = 0; r < v.size(); r += step) {
    auto one = xdr::xdr_to_opaque(v[r]);
    if (one.size() != off[r + 1] - off[r] || memcmp(one.data(), out.data() + off[r], one.size()))
      die("per-record encode differs at " + std::to_string(r));
    T back{};
    xdr::xdr_from_opaque(one, back);
    if (!same(back, v[r])) die("round trip differs at " + std::to_string(r));
  }
  write_file(prefix + ".native", nat.data(), nat.size());
  write_file(prefix + ".heap", heap.b.data(), heap.b.size());
  write_file(prefix + ".xdr", out.data(), out.size());
  write_file(prefix + ".offsets", off.data(), off.size() * 8);
  if (!with_msgs) return;
  // The same records as messages: xdr_to_msg(r) per record (marshal.h:
  // 252-260; mark by message_t::alloc, marshal.cc:15-31), raw_data() of
  // raw_size() bytes each, back to back as msg_sock::output writes them;
  // each message is also read back with xdr_from_msg.
  vector<uint8_t> msgs;
  vector<uint64_t> moff(v.size() + 1, 0);
  msgs.reserve(out.size() + 4 * v.size());
  for (size_t r = 0; r < v.size(); ++r) {
    xdr::msg_ptr m = xdr::xdr_to_msg(v[r]);
    moff[r] = msgs.size();
    msgs.insert(msgs.end(), reinterpret_cast<const uint8_t *>(m->raw_data()),
                reinterpret_cast<const uint8_t *>(m->raw_data()) + m->raw_size());
    if (r % step == 0) {
      T back{};
      xdr::xdr_from_msg(m, back);
      if (!same(back, v[r])) die("xdr_from_msg round trip differs at " + std::to_string(r));
    }
  }
  moff[v.size()] = msgs.size();
  write_file(prefix + ".msgs", msgs.data(), msgs.size());
  write_file(prefix + ".msgoffs", moff.data(), moff.size() * 8);
}

// ------------------------------------------------------------- KAT / errors
static string hex(const uint8_t *p, size_t n) {
  static const char *d = "0123456789abcdef";
  string s;
  for (size_t i = 0; i < n; ++i) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
  return s;
}
static vector<uint8_t> unhex(const string &s) {
  vector<uint8_t> v;
  for (size_t i = 0; i + 1 < s.size(); i += 2) v.push_back(uint8_t(std::stoul(s.substr(i, 2), nullptr, 16)));
  return v;
}
template <typename T> static string enc(const T &t) {
  auto v = xdr::xdr_to_opaque(t);
  return hex(v.data(), v.size());
}
static string json_str(const string &s) {
  string o = "\"";
  for (char c : s) { if (c == '"' || c == '\\') o += '\\'; o += c; }
  return o + "\"";
}

// Decode `h` (hex) as T with the reference; report exception class + what().
template <typename T>
static string try_decode(const string &h, std::function<void(xdr::opaque_vec<> &)> mut = nullptr) {
  auto v = unhex(h);
  xdr::opaque_vec<> m(v.begin(), v.end());
  if (mut) mut(m);
  T t{};
  string cls = "none", what;
  try {
    xdr::xdr_from_opaque(m, t);
  } catch (const xdr::xdr_overflow &e) { cls = "xdr_overflow"; what = e.what(); }
  catch (const xdr::xdr_stack_overflow &e) { cls = "xdr_stack_overflow"; what = e.what(); }
  catch (const xdr::xdr_bad_message_size &e) { cls = "xdr_bad_message_size"; what = e.what(); }
  catch (const xdr::xdr_bad_discriminant &e) { cls = "xdr_bad_discriminant"; what = e.what(); }
  catch (const xdr::xdr_should_be_zero &e) { cls = "xdr_should_be_zero"; what = e.what(); }
  catch (const xdr::xdr_invariant_failed &e) { cls = "xdr_invariant_failed"; what = e.what(); }
  std::ostringstream o;
  o << "{\"input\": \"" << hex(m.data(), m.size()) << "\", \"exception\": \"" << cls
    << "\", \"what\": " << json_str(what) << "}";
  return o.str();
}

static void kat(const string &path) {
  std::ostringstream o;
  o << "{\n";
  // numerics with the tests/marshal.cc:482-490 values
  vector<testns::numerics> nv;
  gen_numerics(1, WG_SEED_NUMERICS, nv);
  o << "  \"numerics_marshal_cc\": \"" << enc(nv[0]) << "\",\n";
  {
    xdr::msg_ptr m = xdr::xdr_to_msg(nv[0]);  // message_t::alloc's mark + the record
    o << "  \"numerics_msg\": \"" << hex(reinterpret_cast<const uint8_t *>(m->raw_data()), m->raw_size())
      << "\",\n";
  }
  // rec128 record 0 of the benchmark stream
  vector<rec128> rv;
  gen_rec128(1, WG_SEED_REC128, 0, rv);
  o << "  \"rec128_0\": \"" << enc(rv[0]) << "\",\n";
  // scalar known answers
  o << "  \"int64_m2\": \"" << enc(int64_t(-2)) << "\",\n";
  o << "  \"float_m0\": \"" << enc(-0.0f) << "\",\n";
  o << "  \"bool_true\": \"" << enc(true) << "\",\n";
  // recvar with lengths 0..7 for every residue mod 4
  for (int bl = 0; bl < 8; ++bl) {
    recvar x{};
    x.id = 0x0102030405060708ULL;
    x.kind = -2;
    x.score = 1.5;
    for (int j = 0; j < bl; ++j) x.blob.push_back(uint8_t(j + 1));
    x.name = string(size_t((bl * 3) % 7), 'h');
    o << "  \"recvar_len" << bl << "\": \"" << enc(x) << "\",\n";
  }
  // SURVEY §8(c) known answers over oracle/x/kat.x.  The union and the
  // xvector alone encode as the one-field structs the plans describe.
  {
    katns::ku u(katns::KRED);
    u.i() = -1;
    katns::ku_rec ur;
    ur.u = u;
    if (enc(u) != enc(ur)) die("kat: union alone != in a struct");
    o << "  \"union_red_m1\": \"" << enc(ur) << "\",\n";
    katns::ku h(katns::KREDDER);
    h.h() = 0x0102030405060708ull;
    katns::ku_rec hr;
    hr.u = h;
    o << "  \"union_redder\": \"" << enc(hr) << "\",\n";
    katns::ku_rec dr;
    dr.u = katns::ku(katns::KREDDEST);  // the default (void) arm
    o << "  \"union_default\": \"" << enc(dr) << "\",\n";
    xdr::xvector<int32_t> xv{1, 2};
    katns::kint_vec kv;
    kv.v = xv;
    if (enc(xv) != enc(kv)) die("kat: xvector alone != in a struct");
    o << "  \"xvector_int_1_2\": \"" << enc(kv) << "\",\n";
    katns::kstruct ks;
    ks.i = -2;
    ks.u = 0x0102030405060708ull;
    ks.d = 1.5;
    ks.blob = {1, 2, 3};
    ks.name = "hello";
    o << "  \"struct_hello\": \"" << enc(ks) << "\",\n";
    // a4: xdr_generic_put checks capacity, not bounds (marshal.h:118-127):
    // past-bound fields encode; their decode throws (types.h:486-489, :539-542)
    auto bounded = [](size_t nb, size_t ns, size_t nv) {
      katns::kbounded b;
      for (size_t j = 0; j < nb; ++j) b.blob.push_back(uint8_t(j + 1));  // std::vector: unchecked
      for (size_t j = 0; j < ns; ++j) static_cast<std::string &>(b.s).push_back(char('a' + j));  // xstring::push_back checks
      for (size_t j = 0; j < nv; ++j) b.v.push_back(int32_t(j + 10));
      return b;
    };
    const katns::kbounded over_all = bounded(65, 9, 3), over_blob = bounded(65, 8, 2),
                          over_s = bounded(64, 9, 2), over_v = bounded(64, 8, 3), in = bounded(64, 8, 2);
    o << "  \"bounded_in\": \"" << enc(in) << "\",\n";
    o << "  \"bounded_over_all\": \"" << enc(over_all) << "\",\n";
    o << "  \"bounded_over_blob\": \"" << enc(over_blob) << "\",\n";
    o << "  \"bounded_over_s\": \"" << enc(over_s) << "\",\n";
    o << "  \"bounded_over_v\": \"" << enc(over_v) << "\",\n";
  }
  // rpc: one of each arm
  vector<xdr::rpc_msg> pv;
  gen_rpc(64, WG_SEED_RPC, pv);
  o << "  \"rpc_first64\": [";
  for (size_t i = 0; i < pv.size(); ++i) o << (i ? ", " : "") << "\"" << enc(pv[i]) << "\"";
  o << "],\n";

  // ---- error cases: exception class + what() from the reference decoder
  o << "  \"errors\": {\n";
  string good_nv = enc(nv[0]);
  vector<recvar> vv;
  gen_recvar(4, WG_SEED_RECVAR, vv);
  recvar odd{};
  odd.blob = {1, 2, 3};  // 3 bytes -> one pad byte
  odd.name = "hello";
  string good_rv = enc(odd);
  o << "    \"numerics_ok\": " << try_decode<testns::numerics>(good_nv) << ",\n";
  o << "    \"numerics_short\": " << try_decode<testns::numerics>(good_nv.substr(0, 80)) << ",\n";
  o << "    \"numerics_trailing\": " << try_decode<testns::numerics>(good_nv + "00000000") << ",\n";
  o << "    \"numerics_not_mult4\": " << try_decode<testns::numerics>(good_nv + "00") << ",\n";
  o << "    \"numerics_bool2\": "
    << try_decode<testns::numerics>(good_nv, [](xdr::opaque_vec<> &m) { m[3] = 2; }) << ",\n";
  o << "    \"numerics_enum99_novalidate\": "
    << try_decode<testns::numerics>(good_nv, [](xdr::opaque_vec<> &m) { m[43] = 99; }) << ",\n";
  o << "    \"numerics_enum99_validate\": "
    << try_decode<testns_v::numerics>(good_nv, [](xdr::opaque_vec<> &m) { m[43] = 99; }) << ",\n";
  o << "    \"recvar_ok\": " << try_decode<recvar>(good_rv) << ",\n";
  // blob is 01020300: make the pad byte nonzero
  o << "    \"recvar_nonzero_pad\": "
    << try_decode<recvar>(good_rv, [](xdr::opaque_vec<> &m) { m[19] = 0x7f; }) << ",\n";
  o << "    \"recvar_blob_over_bound\": "
    << try_decode<recvar>(good_rv, [](xdr::opaque_vec<> &m) {
         // claim 260 bytes (> 256) and supply them
         xdr::opaque_vec<> n(m.begin(), m.begin() + 12);  // id kind
         uint32_t L = 260;
         n.push_back(uint8_t(L >> 24)); n.push_back(uint8_t(L >> 16));
         n.push_back(uint8_t(L >> 8)); n.push_back(uint8_t(L));
         for (uint32_t j = 0; j < L; ++j) n.push_back(1);
         for (int j = 0; j < 12; ++j) n.push_back(0);
         m = n;
       }) << ",\n";
  o << "    \"recvar_name_over_bound\": "
    << try_decode<recvar>(good_rv, [](xdr::opaque_vec<> &m) {
         xdr::opaque_vec<> n(m.begin(), m.begin() + 20);  // id kind blob(3)
         uint32_t L = 68;
         n.push_back(0); n.push_back(0); n.push_back(0); n.push_back(uint8_t(L));
         for (uint32_t j = 0; j < L; ++j) n.push_back('x');
         for (int j = 0; j < 8; ++j) n.push_back(0);
         m = n;
       }) << ",\n";
  o << "    \"recvar_len_past_end\": "
    << try_decode<recvar>(good_rv, [](xdr::opaque_vec<> &m) { m[15] = 200; }) << ",\n";
  string good_rpc = enc(pv[0]);
  o << "    \"rpc_ok\": " << try_decode<xdr::rpc_msg>(good_rpc) << ",\n";
  o << "    \"rpc_bad_mtype\": "
    << try_decode<xdr::rpc_msg>(good_rpc, [](xdr::opaque_vec<> &m) { m[7] = 7; }) << ",\n";
  {
    // a MSG_DENIED reply with a bad reject_stat
    xdr::rpc_msg d{};
    d.xid = 9;
    d.body.mtype(xdr::REPLY);
    d.body.rbody().stat(xdr::MSG_DENIED);
    d.body.rbody().rreply().stat(xdr::AUTH_ERROR);
    d.body.rbody().rreply().rj_why() = xdr::auth_stat(3);
    string h = enc(d);
    o << "    \"rpc_denied_ok\": " << try_decode<xdr::rpc_msg>(h) << ",\n";
    o << "    \"rpc_bad_reject_stat\": "
      << try_decode<xdr::rpc_msg>(h, [](xdr::opaque_vec<> &m) { m[15] = 5; }) << ",\n";
    o << "    \"rpc_bad_reply_stat\": "
      << try_decode<xdr::rpc_msg>(h, [](xdr::opaque_vec<> &m) { m[11] = 2; }) << ",\n";
  }
  {
    // vecrec: id, vals<16> = {5, -6}, opt = {7, 8}, pairs<8> = {(9, true)}, flag
    vecrec x{};
    x.id = 1;
    x.vals = {5, -6};
    x.opt.activate() = ::mismatch_info{7, 8};
    x.pairs.resize(1);
    x.pairs[0].h = 9;
    x.pairs[0].b = true;
    x.flag = false;
    const string h = enc(x);
    // layout: id @0, vals count @4, vals @8..16, opt count @16, opt @20..28,
    // pairs count @28, pair @32..44, flag @44
    o << "    \"vecrec_ok\": " << try_decode<vecrec>(h) << ",\n";
    o << "    \"vecrec_vals_over_bound\": "
      << try_decode<vecrec>(h, [](xdr::opaque_vec<> &m) { m[7] = 17; }) << ",\n";
    o << "    \"vecrec_pointer_two\": "
      << try_decode<vecrec>(h, [](xdr::opaque_vec<> &m) { m[19] = 2; }) << ",\n";
    o << "    \"vecrec_pairs_past_end\": "
      << try_decode<vecrec>(h, [](xdr::opaque_vec<> &m) { m[31] = 3; }) << ",\n";
    o << "    \"vecrec_bool2\": "
      << try_decode<vecrec>(h, [](xdr::opaque_vec<> &m) { m[43] = 2; }) << ",\n";
  }
  {
    // the past-bound encodes of kat.x kbounded (above), decoded
    auto bounded = [](size_t nb, size_t ns, size_t nv) {
      katns::kbounded b;
      for (size_t j = 0; j < nb; ++j) b.blob.push_back(uint8_t(j + 1));
      for (size_t j = 0; j < ns; ++j) static_cast<std::string &>(b.s).push_back(char('a' + j));  // xstring::push_back checks
      for (size_t j = 0; j < nv; ++j) b.v.push_back(int32_t(j + 10));
      return enc(b);
    };
    o << "    \"kbounded_in\": " << try_decode<katns::kbounded>(bounded(64, 8, 2)) << ",\n";
    o << "    \"kbounded_over_blob\": " << try_decode<katns::kbounded>(bounded(65, 8, 2)) << ",\n";
    o << "    \"kbounded_over_s\": " << try_decode<katns::kbounded>(bounded(64, 9, 2)) << ",\n";
    o << "    \"kbounded_over_v\": " << try_decode<katns::kbounded>(bounded(64, 8, 3)) << ",\n";
    o << "    \"kbounded_over_all\": " << try_decode<katns::kbounded>(bounded(65, 9, 3)) << "\n";
  }
  o << "  }\n}\n";
  std::ofstream f(path);
  f << o.str();
}

// ------------------------------------------------------------- bench mode
template <typename T>
static void bench_one(const char *name, const vector<T> &v, int threads, int reps) {
  vector<uint64_t> off(v.size() + 1, 0);
  for (size_t r = 0; r < v.size(); ++r) off[r + 1] = off[r] + xdr::xdr_size(v[r]);
  vector<uint8_t> out(off.back());
  vector<T> back(v.size());
  auto run = [&](auto &&body) {
    vector<std::thread> th;
    size_t n = v.size();
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] { body(n * t / threads, n * (t + 1) / threads); });
    for (auto &x : th) x.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  };
  auto encode = [&](size_t a, size_t b) {
    xdr::xdr_put p(out.data() + off[a], out.data() + off[b]);
    for (size_t r = a; r < b; ++r) archive(p, v[r]);
  };
  auto decode = [&](size_t a, size_t b) {
    xdr::xdr_get g(out.data() + off[a], out.data() + off[b]);
    for (size_t r = a; r < b; ++r) archive(g, back[r]);
    g.done();
  };
  auto per_record = [&](size_t a, size_t b) {
    for (size_t r = a; r < b; ++r) {
      auto m = xdr::xdr_to_opaque(v[r]);
      memcpy(out.data() + off[r], m.data(), m.size());
    }
  };
  run(encode);  // pre-fault
  run(decode);
  vector<double> te, td, tp;
  for (int i = 0; i < reps; ++i) {
    te.push_back(run(encode));
    td.push_back(run(decode));
    tp.push_back(run(per_record));
  }
  std::sort(te.begin(), te.end());
  std::sort(td.begin(), td.end());
  std::sort(tp.begin(), tp.end());
  double gib = double(off.back()) / (1024.0 * 1024 * 1024);
  printf("{\"schema\": \"%s\", \"records\": %zu, \"xdr_bytes\": %llu, \"threads\": %d, "
         "\"reps\": %d, \"encode_s_best\": %.6f, \"encode_s_median\": %.6f, "
         "\"decode_s_best\": %.6f, \"decode_s_median\": %.6f, \"to_opaque_s_best\": %.6f, "
         "\"encode_gib_s\": %.4f, \"decode_gib_s\": %.4f, \"to_opaque_gib_s\": %.4f, "
         "\"encode_decode_gib_s\": %.4f}\n",
         name, v.size(), (unsigned long long)off.back(), threads, reps, te[0], te[reps / 2],
         td[0], td[reps / 2], tp[0], gib / te[0], gib / td[0], gib / tp[0],
         2 * gib / (te[0] + td[0]));
}

// ------------------------------------------------------------ RPC headers
// ref_golden rpc <stream> <offsets> <procs> <xids|-> <outprefix>
//
// Every message [off[k], off[k+1]) of the stream goes through the REAL
// reference paths, compiled from /root/reference against the generated
// xdrpp/rpc_msg.hh (oracle/Makefile):
//  * the header decode, archive(g, hdr) with xdr_get over the message body
//    (xdrpp/marshal.h:142-211), for the fields of xdrg_rpc_hdr;
//  * the server: rpc_server_base::dispatch (xdrpp/server.cc:78-117) with a
//    service registered for every (prog, vers) of the procedure table; a
//    service's process() is srpc_service::process (xdrpp/srpc.h:121-128)
//    whose call_dispatch knows the table's procedures.  The reply dispatch
//    sends -- built by the real rpc_*_msg, server.cc:8-67 -- is the
//    fixture's reply, and its words name the action;
//  * the client: the real check_call_hdr (xdrpp/rpc_msg.cc:114-131) + the
//    xid test of srpc.h:61-66.
// Writes <outprefix>.hdrs / .chk (xdrg_rpc_hdr per message, server / client
// classification) and .replies / .replyoffs.
#include <xdrpp/exception.h>
#include <xdrpp/server.h>

#include <iostream>
#include <map>
#include <set>

static vector<uint8_t> slurp(const string &path) {
  FILE *f = fopen(path.c_str(), "rb");
  if (!f) die("cannot open " + path);
  vector<uint8_t> b;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + k);
  fclose(f);
  return b;
}

namespace rpcref {
// srpc_service::process (srpc.h:121-128) for an interface whose
// call_dispatch has a case for each procedure in `procs`.
struct table_service : xdr::service_base {
  std::set<uint32_t> procs;
  bool *dispatched;
  table_service(uint32_t prog, uint32_t vers, std::set<uint32_t> p, bool *d)
      : service_base(prog, vers), procs(std::move(p)), dispatched(d) {}
  void process(void *, xdr::rpc_msg &hdr, xdr::xdr_get &, cb_t reply) override {
    if (!check_call(hdr)) reply(nullptr);
    if (procs.count(hdr.body.cbody().proc)) {
      *dispatched = true;  // call_dispatch's case: the procedure runs
      return;
    }
    reply(xdr::rpc_accepted_error_msg(hdr.xid, xdr::PROC_UNAVAIL));
  }
};
struct table_server : xdr::rpc_server_base {
  void add(table_service *s) { register_service_base(s); }
};

static uint8_t err_code(const std::exception &e, const string &w, uint32_t *site) {
  *site = 0;
  if (dynamic_cast<const xdr::xdr_bad_discriminant *>(&e)) {
    if (w.find("reply_body") != string::npos) *site = 1;
    else if (w.find("rejected_reply") != string::npos) *site = 2;
    return XDRG_ERR_BAD_DISCRIMINANT;
  }
  if (dynamic_cast<const xdr::xdr_should_be_zero *>(&e)) return XDRG_ERR_NONZERO_PAD;
  if (w == "xvector overflow") return XDRG_ERR_XVECTOR_BOUND;
  if (dynamic_cast<const xdr::xdr_overflow *>(&e)) return XDRG_ERR_OVERFLOW_GET;
  if (dynamic_cast<const xdr::xdr_bad_message_size *>(&e)) return XDRG_ERR_SIZE_NOT_MULT4;
  die("unexpected exception " + w);
  return 0;
}
}  // namespace rpcref

static void rpc_mode(const string &sp, const string &op, const string &pp, const string &xp,
                     const string &pre) {
  vector<uint8_t> sb = slurp(sp), ob = slurp(op), pb = slurp(pp), xb;
  if (xp != "-") xb = slurp(xp);
  // 4-byte aligned copy of the stream (xdr_get asserts an aligned start)
  vector<uint32_t> words((sb.size() + 3) / 4);
  memcpy(words.data(), sb.data(), sb.size());
  const uint8_t *s = reinterpret_cast<const uint8_t *>(words.data());
  const uint64_t *off = reinterpret_cast<const uint64_t *>(ob.data());
  const size_t n = ob.size() / 8 - 1;
  const xdrg_rpc_proc *pt = reinterpret_cast<const xdrg_rpc_proc *>(pb.data());
  const size_t np = pb.size() / sizeof(xdrg_rpc_proc);
  std::map<std::pair<uint32_t, uint32_t>, std::set<uint32_t>> ifaces;
  for (size_t i = 0; i < np; ++i) {
    auto &procs = ifaces[{pt[i].prog, pt[i].vers}];
    if (!(pt[i].flags & XDRG_RPC_PROC_IFACE_ONLY)) procs.insert(pt[i].proc);
  }
  bool dispatched = false;
  rpcref::table_server server;
  for (auto &f : ifaces) server.add(new rpcref::table_service(f.first.first, f.first.second, f.second, &dispatched));
  std::streambuf *cerr_buf = std::cerr.rdbuf(nullptr);  // dispatch's diagnostics
  vector<xdrg_rpc_hdr> hs(n), cs(n);
  vector<uint8_t> rep;
  vector<uint64_t> roff(n + 1, 0);
  for (size_t k = 0; k < n; ++k) {
    const uint64_t m0 = off[k], m1 = off[k + 1];
    xdrg_rpc_hdr h;
    memset(&h, 0, sizeof h);
    h.end = m1;
    xdr::rpc_msg hdr;
    uint8_t err = 0;
    uint32_t site = 0;
    try {
      xdr::xdr_get g(s + m0 + 4, s + m1);
      archive(g, hdr);
      h.body_off = reinterpret_cast<const uint8_t *>(g.p_) - s;
    } catch (const std::exception &e) {
      err = rpcref::err_code(e, e.what(), &site);
    }
    if (!err) {
      h.xid = hdr.xid;
      h.mtype = uint8_t(hdr.body.mtype());
      if (hdr.body.mtype() == xdr::CALL) {
        const xdr::call_body &cb = hdr.body.cbody();
        h.w[XDRG_RPC_W_RPCVERS] = cb.rpcvers; h.w[XDRG_RPC_W_PROG] = cb.prog;
        h.w[XDRG_RPC_W_VERS] = cb.vers; h.w[XDRG_RPC_W_PROC] = cb.proc;
        h.w[XDRG_RPC_W_CRED_FLAVOR] = uint32_t(cb.cred.flavor);
        h.w[XDRG_RPC_W_VERF_FLAVOR] = uint32_t(cb.verf.flavor);
        h.cred_len = uint32_t(cb.cred.body.size());
        h.verf_len = uint32_t(cb.verf.body.size());
      } else {
        const xdr::reply_body &rb = hdr.body.rbody();
        h.w[XDRG_RPC_W_REPLY_STAT] = uint32_t(rb.stat());
        if (rb.stat() == xdr::MSG_ACCEPTED) {
          h.w[XDRG_RPC_W_VERF_FLAVOR] = uint32_t(rb.areply().verf.flavor);
          h.verf_len = uint32_t(rb.areply().verf.body.size());
          h.w[XDRG_RPC_W_STAT] = uint32_t(rb.areply().reply_data.stat());
          if (rb.areply().reply_data.stat() == xdr::PROG_MISMATCH) {
            h.w[XDRG_RPC_W_LOW] = rb.areply().reply_data.mismatch_info().low;
            h.w[XDRG_RPC_W_HIGH] = rb.areply().reply_data.mismatch_info().high;
          }
        } else {
          h.w[XDRG_RPC_W_STAT] = uint32_t(rb.rreply().stat());
          if (rb.rreply().stat() == xdr::RPC_MISMATCH) {
            h.w[XDRG_RPC_W_LOW] = rb.rreply().mismatch_info().low;
            h.w[XDRG_RPC_W_HIGH] = rb.rreply().mismatch_info().high;
          } else {
            h.w[XDRG_RPC_W_WHY] = uint32_t(rb.rreply().rj_why());
          }
        }
      }
    } else {
      h.err = err;
      h.w[0] = site;
    }
    // ---- server: the real rpc_server_base::dispatch
    xdrg_rpc_hdr sv = h;
    xdr::msg_ptr m = xdr::message_t::alloc(m1 - m0 - 4);
    memcpy(m->data(), s + m0 + 4, m1 - m0 - 4);
    xdr::msg_ptr reply;
    dispatched = false;
    server.dispatch(nullptr, std::move(m), [&](xdr::msg_ptr r) { reply = std::move(r); });
    if (dispatched) {
      sv.action = XDRG_RPC_DISPATCH;
    } else if (reply) {  // words: xid REPLY reply_stat ...
      auto w = [&](size_t i) { return __builtin_bswap32(reinterpret_cast<const uint32_t *>(reply->data())[i]); };
      if (w(2) == xdr::MSG_DENIED) {
        if (w(3) != xdr::RPC_MISMATCH) die("unexpected denied reply");
        sv.action = XDRG_RPC_RPC_MISMATCH;
      } else {
        switch (w(5)) {  // accept_stat after the AUTH_NONE verifier
        case xdr::PROG_UNAVAIL: sv.action = XDRG_RPC_PROG_UNAVAIL; break;
        case xdr::PROG_MISMATCH:
          sv.action = XDRG_RPC_PROG_MISMATCH;
          sv.w[XDRG_RPC_W_LOW] = w(6);
          sv.w[XDRG_RPC_W_HIGH] = w(7);
          break;
        case xdr::PROC_UNAVAIL: sv.action = XDRG_RPC_PROC_UNAVAIL; break;
        case xdr::GARBAGE_ARGS: sv.action = XDRG_RPC_GARBAGE_ARGS; break;
        default: die("unexpected accepted reply");
        }
      }
    } else {  // dispatch dropped the message
      sv.action = err ? XDRG_RPC_DROP_MALFORMED : XDRG_RPC_DROP_NONCALL;
    }
    hs[k] = sv;
    if (reply)
      rep.insert(rep.end(), reinterpret_cast<const uint8_t *>(reply->raw_data()),
                 reinterpret_cast<const uint8_t *>(reply->raw_data()) + reply->raw_size());
    roff[k + 1] = rep.size();
    // ---- client: archive(g, hdr); the real check_call_hdr; xid (srpc.h:61-66)
    xdrg_rpc_hdr cl = h;
    if (err) {
      cl.action = XDRG_RPCR_MALFORMED;
    } else {
      try {
        xdr::check_call_hdr(hdr);
        cl.action = XDRG_RPCR_OK;
      } catch (const xdr::xdr_call_error &e) {
        switch (e.stat_.type_) {
        case xdr::rpc_call_stat::ACCEPT_STAT: cl.action = XDRG_RPCR_ACCEPT_STAT; break;
        case xdr::rpc_call_stat::AUTH_STAT: cl.action = XDRG_RPCR_AUTH_STAT; break;
        case xdr::rpc_call_stat::RPCVERS_MISMATCH: cl.action = XDRG_RPCR_RPCVERS_MISMATCH; break;
        default: die("unexpected call error");
        }
      } catch (const xdr::xdr_runtime_error &) {
        cl.action = XDRG_RPCR_NOT_REPLY;  // "call received when reply expected"
      }
    }
    if (cl.action == XDRG_RPCR_OK && !xb.empty() &&
        reinterpret_cast<const uint32_t *>(xb.data())[k] != hdr.xid)
      cl.action = XDRG_RPCR_BAD_XID;
    cs[k] = cl;
  }
  std::cerr.rdbuf(cerr_buf);
  write_file(pre + ".hdrs", hs.data(), hs.size() * sizeof(xdrg_rpc_hdr));
  write_file(pre + ".chk", cs.data(), cs.size() * sizeof(xdrg_rpc_hdr));
  write_file(pre + ".replies", rep.data(), rep.size());
  write_file(pre + ".replyoffs", roff.data(), roff.size() * 8);
  // the auth-error reply has no dispatch route; one known answer of it
  xdr::msg_ptr ae = xdr::rpc_auth_error_msg(0x01020304u, xdr::auth_stat(5));
  write_file(pre + ".autherr", ae->raw_data(), ae->raw_size());
}

// ------------------------------------------------------------ depths
// ref_golden depths <schema> <n> <out>: per record the smallest limit L for
// which the REAL xdr::check_xdr_depth(r, L) holds (xdrpp/depth_checker.h).
#include <xdrpp/depth_checker.h>

template <typename T> static void depths_of(const vector<T> &v, const string &out) {
  vector<uint32_t> d(v.size());
  for (size_t r = 0; r < v.size(); ++r) {
    uint32_t L = 0;
    while (!xdr::check_xdr_depth(v[r], L)) ++L;
    d[r] = L;
  }
  write_file(out, d.data(), d.size() * 4);
}

// frame <stream file> <maxmsglen> <out.json>: the messages of a stream as
// the REAL read_message (srpc.cc:29-55) reads them from a file descriptor,
// message after message, with msg_sock's length rule in front of each
// (msgsock.cc:97-111: a message longer than maxmsglen is rejected).  Out:
// {"offsets": [mark of each message, then where the framing stopped],
//  "what": the exception's what() or "too long" or null at a clean end}.
// A clean end is the stream's end reached exactly at a mark.
#include <fcntl.h>
#include <unistd.h>
#include <xdrpp/srpc.h>

static void frame_mode(const string &in, uint64_t maxlen, const string &out) {
  const int fd = open(in.c_str(), O_RDONLY);
  if (fd < 0) die("open " + in);
  const off_t len = lseek(fd, 0, SEEK_END);
  lseek(fd, 0, SEEK_SET);
  std::ostringstream o;
  o << "{\"offsets\": [";
  uint64_t pos = 0;
  string what = "null";
  for (bool first = true;; first = false) {
    o << (first ? "" : ", ") << pos;
    if (pos == static_cast<uint64_t>(len)) break;
    uint32_t raw = 0;
    if (pread(fd, &raw, 4, pos) == 4) {  // msg_sock's rule needs the size first
      const uint32_t v = xdr::swap32le(raw);
      if (!(raw & 3) && (v & 0x80000000u) && (v & 0x7fffffffu) > maxlen) { what = "\"too long\""; break; }
    }
    try {
      xdr::msg_ptr m = xdr::read_message(fd);
      pos += m->raw_size();
    } catch (const std::exception &e) {
      what = string("\"") + e.what() + "\"";
      break;
    }
  }
  o << "], \"what\": " << what << "}\n";
  close(fd);
  std::ofstream f(out);
  f << o.str();
}

// ---- success replies: xdr_to_msg(rpc_success_hdr(xid), res) (the reply
// srpc_service::dispatch sends, xdrpp/srpc.h:152, header xdrpp/server.h:
// 27-49) for rec128 results r (the config-2 generator) and xid_r = r *
// 2654435761, back to back; and the reference's own byte assertion
// (tests/arpc.cc:35-43): xdr_to_msg(rpc_msg(7, REPLY)) == xdr_to_msg(
// rpc_success_hdr(7)), both messages written after it.
static void success_mode(size_t n, const string &pre) {
  vector<rec128> v;
  gen_rec128(n, WG_SEED_REC128, 0, v);
  std::vector<uint8_t> out;
  for (size_t r = 0; r < n; ++r) {
    const uint32_t xid = static_cast<uint32_t>(r * 2654435761u);
    xdr::msg_ptr m = xdr::xdr_to_msg(xdr::rpc_success_hdr(xid), v[r]);
    const uint8_t *b = reinterpret_cast<const uint8_t *>(m->raw_data());
    out.insert(out.end(), b, b + m->raw_size());
  }
  write_file(pre + ".msgs", out.data(), out.size());
  xdr::msg_ptr m1(xdr::xdr_to_msg(xdr::rpc_msg(7, xdr::REPLY)));
  xdr::msg_ptr m2(xdr::xdr_to_msg(xdr::rpc_success_hdr(7)));
  if (m1->size() != m2->size() || memcmp(m1->data(), m2->data(), m1->size()))
    die("rpc_msg(7, REPLY) and rpc_success_hdr(7) differ");
  write_file(pre + ".hdr7", m2->raw_data(), m2->raw_size());
}

int main(int argc, char **argv) {
  if (argc < 2) die("usage: gen|kat|bench|rpc|frame|success ...");
  if (string(argv[1]) == "success") {
    if (argc != 4) die("success <n> <outprefix>");
    success_mode(std::stoull(argv[2]), argv[3]);
    return 0;
  }
  string mode = argv[1];
  if (mode == "frame") {
    if (argc != 5) die("frame <stream> <maxmsglen> <out.json>");
    frame_mode(argv[2], std::stoull(argv[3]), argv[4]);
    return 0;
  }
  if (mode == "kat") {
    if (argc != 3) die("kat <out.json>");
    kat(argv[2]);
    return 0;
  }
  if (mode == "rpc") {
    if (argc != 7) die("rpc <stream> <offsets> <procs> <xids|-> <outprefix>");
    rpc_mode(argv[2], argv[3], argv[4], argv[5], argv[6]);
    return 0;
  }
  if (argc < 4) die("missing args");
  string schema = argv[2];
  size_t n = std::stoull(argv[3]);
  if (mode == "gen") {
    if (argc != 5 && argc != 6) die("gen <schema> <n> <prefix> [nomsgs]");
    string pre = argv[4];
    const bool wm = !(argc == 6 && string(argv[5]) == "nomsgs");
    if (schema == "numerics") { vector<testns::numerics> v; gen_numerics(n, WG_SEED_NUMERICS, v); emit(v, pre, wm); }
    else if (schema == "rec128") { vector<rec128> v; gen_rec128(n, WG_SEED_REC128, 0, v); emit(v, pre, wm); }
    else if (schema == "rec128_mgpu") { vector<rec128> v; gen_rec128(n, WG_SEED_REC128_MGPU, 0, v); emit(v, pre, wm); }
    else if (schema == "recvar") { vector<recvar> v; gen_recvar(n, WG_SEED_RECVAR, v); emit(v, pre, wm); }
    else if (schema == "vecrec") { vector<vecrec> v; gen_vecrec(n, WG_SEED_VECREC, v); emit(v, pre, wm); }
    else if (schema == "containertest") { vector<testns::containertest> v; gen_containertest(n, WG_SEED_CONTAINERTEST, v); emit(v, pre, wm); }
    else if (schema == "rpc") { vector<xdr::rpc_msg> v; gen_rpc(n, WG_SEED_RPC, v); emit(v, pre, wm); }
    else if (schema == "rp_list") { vector<xdr::rp__list> v; gen_rp_list(n, WG_SEED_RP_LIST, v); emit(v, pre, wm); }
    else die("unknown schema " + schema);
    return 0;
  }
  if (mode == "depths") {
    if (argc != 5) die("depths <schema> <n> <out>");
    string o = argv[4];
    if (schema == "numerics") { vector<testns::numerics> v; gen_numerics(n, WG_SEED_NUMERICS, v); depths_of(v, o); }
    else if (schema == "rec128") { vector<rec128> v; gen_rec128(n, WG_SEED_REC128, 0, v); depths_of(v, o); }
    else if (schema == "recvar") { vector<recvar> v; gen_recvar(n, WG_SEED_RECVAR, v); depths_of(v, o); }
    else if (schema == "vecrec") { vector<vecrec> v; gen_vecrec(n, WG_SEED_VECREC, v); depths_of(v, o); }
    else if (schema == "containertest") { vector<testns::containertest> v; gen_containertest(n, WG_SEED_CONTAINERTEST, v); depths_of(v, o); }
    else if (schema == "rpc") { vector<xdr::rpc_msg> v; gen_rpc(n, WG_SEED_RPC, v); depths_of(v, o); }
    else if (schema == "rp_list") { vector<xdr::rp__list> v; gen_rp_list(n, WG_SEED_RP_LIST, v); depths_of(v, o); }
    else die("unknown schema " + schema);
    return 0;
  }
  if (mode == "bench") {
    if (argc != 6) die("bench <schema> <n> <threads> <reps>");
    int threads = atoi(argv[4]), reps = atoi(argv[5]);
    if (schema == "rec128") { vector<rec128> v; gen_rec128(n, WG_SEED_REC128, 0, v); bench_one("rec128", v, threads, reps); }
    else if (schema == "numerics") { vector<testns::numerics> v; gen_numerics(n, WG_SEED_NUMERICS, v); bench_one("numerics", v, threads, reps); }
    else if (schema == "recvar") { vector<recvar> v; gen_recvar(n, WG_SEED_RECVAR, v); bench_one("recvar", v, threads, reps); }
    else if (schema == "vecrec") { vector<vecrec> v; gen_vecrec(n, WG_SEED_VECREC, v); bench_one("vecrec", v, threads, reps); }
    else if (schema == "containertest") { vector<testns::containertest> v; gen_containertest(n, WG_SEED_CONTAINERTEST, v); bench_one("containertest", v, threads, reps); }
    else if (schema == "rpc") { vector<xdr::rpc_msg> v; gen_rpc(n, WG_SEED_RPC, v); bench_one("rpc", v, threads, reps); }
    else if (schema == "rp_list") { vector<xdr::rp__list> v; gen_rp_list(n, WG_SEED_RP_LIST, v); bench_one("rp_list", v, threads, reps); }
    else die("unknown schema " + schema);
    return 0;
  }
  die("unknown mode " + mode);
}
