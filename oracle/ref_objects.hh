// ORACLE / TEST INFRASTRUCTURE ONLY.
//
// C++ record objects of the benchmark schemas -- genuine xdrc-generated
// types (oracle/ref_types.hh) -- built from the synthetic generator
// (oracle/workload_gen.h), their staged device layout, and equality
// helpers.  Shared by ref_golden.cc and the C++ drop-in test
// (tests/cpp/dropin_test.cc).
#ifndef XDRG_REF_OBJECTS_HH
#define XDRG_REF_OBJECTS_HH
#include "ref_types.hh"
#include "workload_gen.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static_assert(sizeof(st_rp_list) == 72, "rp_list staged node");

namespace refobj {
using std::size_t;
using std::string;
using std::vector;

[[maybe_unused]] static void die(const string &m) {
  fprintf(stderr, "ref_golden: %s\n", m.c_str());
  exit(2);
}
template <typename T> [[maybe_unused]] static T bits_as(uint64_t v) {
  T t;
  memcpy(&t, &v, sizeof(T));
  return t;
}
[[maybe_unused]] static void write_file(const string &path, const void *p, size_t n) {
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) die("cannot open " + path);
  if (n && fwrite(p, 1, n, f) != n) die("short write " + path);
  fclose(f);
}

// ------------------------------------------------------------ generators
[[maybe_unused]] static void gen_numerics(size_t n, uint64_t seed, vector<testns::numerics> &v) {
  v.resize(n);
  for (size_t r = 0; r < n; ++r) {
    testns::numerics &x = v[r];
    memset(&x, 0, sizeof x);  // padding bytes are zero in the fixture
    uint64_t d[8];
    for (int k = 0; k < 8; ++k) d[k] = wg_draw(seed, r * 8 + k);
    x.b = d[0] & 1;
    x.i1 = (int32_t)(uint32_t)d[1];
    x.i2 = (uint32_t)d[2];
    x.i3 = (int64_t)d[3];
    x.i4 = d[4];
    x.f1 = bits_as<float>((uint32_t)d[5]);
    x.f2 = bits_as<double>(d[6]);
    x.e1 = testns::other_color(d[7] % 3);
    if (r == 0) {  // tests/marshal.cc:482-490
      x.b = false;
      x.i1 = 0x7eeeeeee;
      x.i2 = 0xffffffff;
      x.i3 = UINT64_C(0x7ddddddddddddddd);
      x.i4 = UINT64_C(0xfccccccccccccccc);
      x.f1 = 3.141592654;
      x.f2 = 2.71828182846;
      x.e1 = testns::REDDER;
    }
  }
}

[[maybe_unused]] static void gen_rec128(size_t n, uint64_t seed, uint64_t first, vector<rec128> &v) {
  v.resize(n);
  for (size_t r = 0; r < n; ++r) {
    uint64_t g = first + r, d[20];
    for (int k = 0; k < 20; ++k) d[k] = wg_draw(seed, g * 20 + k);
    rec128 &x = v[r];
    int32_t *a = &x.a0;
    for (int k = 0; k < 8; ++k) a[k] = (int32_t)(uint32_t)d[k];
    uint64_t *u = &x.u0;
    for (int k = 0; k < 6; ++k) u[k] = d[8 + k];
    double *dd = &x.d0;
    for (int k = 0; k < 6; ++k) dd[k] = bits_as<double>(d[14 + k]);
  }
}

[[maybe_unused]] static void gen_recvar(size_t n, uint64_t seed, vector<recvar> &v) {
  v.resize(n);
  const uint64_t ps = seed ^ WG_PAYLOAD_XOR;
  for (size_t r = 0; r < n; ++r) {
    uint64_t d[5];
    for (int k = 0; k < 5; ++k) d[k] = wg_draw(seed, r * 5 + k);
    recvar &x = v[r];
    x.id = d[0];
    x.kind = (int32_t)(uint32_t)d[1];
    uint32_t bl = d[2] % 257, nl = d[3] % 65;
    x.score = bits_as<double>(d[4]);
    x.blob.resize(bl);
    for (uint32_t j = 0; j < bl; ++j) x.blob[j] = wg_byte(ps, r * 40 + j / 8, j);
    string s(nl, '\0');
    for (uint32_t j = 0; j < nl; ++j)
      s[j] = char(0x61 + wg_byte(ps, r * 40 + 32 + j / 8, j) % 26);
    x.name = s;
  }
}

// vecrec: draws d[0..5] = draw(seed, 6r + k); element values from the
// payload stream draw(seed ^ XOR, 32r + j)
[[maybe_unused]] static void gen_vecrec(size_t n, uint64_t seed, vector<vecrec> &v) {
  v.resize(n);
  const uint64_t ps = seed ^ WG_PAYLOAD_XOR;
  for (size_t r = 0; r < n; ++r) {
    uint64_t d[6];
    for (int k = 0; k < 6; ++k) d[k] = wg_draw(seed, r * 6 + k);
    vecrec &x = v[r];
    x.id = (uint32_t)d[0];
    const uint32_t nv = d[1] % 17, np = d[3] % 9;
    x.vals.resize(nv);
    for (uint32_t j = 0; j < nv; ++j) x.vals[j] = (int32_t)(uint32_t)wg_draw(ps, r * 32 + j);
    if (d[2] & 1) {
      const uint64_t w = wg_draw(ps, r * 32 + 16);
      x.opt.activate() = ::mismatch_info{(uint32_t)w, (uint32_t)(w >> 32)};
    } else {
      x.opt.reset();
    }
    x.pairs.resize(np);
    for (uint32_t j = 0; j < np; ++j) {
      x.pairs[j].h = (int64_t)wg_draw(ps, r * 32 + 17 + j);
      x.pairs[j].b = (d[5] >> j) & 1;
    }
    x.flag = (d[4] >> 8) & 1;
  }
}

// containertest (tests/xdrtest.x:129-132): d[0..3] = draw(seed, 4r + k);
// nu = d0 % 9 elements, element j the f12 arm if bit j of d1 is set (else
// f4), its int from payload word 32r + j, its double's bits from word
// 32r + 8 + j; |sarr[0]| = d2 % 33, |sarr[1]| = (d2 >> 32) % 33, letters
// from payload words 32r + 16 + k/8 and 32r + 21 + k/8
[[maybe_unused]] static void gen_containertest(size_t n, uint64_t seed, vector<testns::containertest> &v) {
  v.resize(n);
  const uint64_t ps = seed ^ WG_PAYLOAD_XOR;
  for (size_t r = 0; r < n; ++r) {
    uint64_t d[4];
    for (int k = 0; k < 4; ++k) d[k] = wg_draw(seed, r * 4 + k);
    testns::containertest &x = v[r];
    const uint32_t nu = d[0] % 9;
    x.uvec.resize(nu);
    for (uint32_t j = 0; j < nu; ++j) {
      const int32_t i = (int32_t)(uint32_t)wg_draw(ps, r * 32 + j);
      if ((d[1] >> j) & 1) {
        x.uvec[j].which(12);
        x.uvec[j].f12().i = i;
        x.uvec[j].f12().d = bits_as<double>(wg_draw(ps, r * 32 + 8 + j));
      } else {
        x.uvec[j].which(4);
        x.uvec[j].f4().i = i;
      }
    }
    const uint32_t len[2] = {uint32_t(d[2] % 33), uint32_t((d[2] >> 32) % 33)};
    for (int k = 0; k < 2; ++k) {
      string s(len[k], '\0');
      for (uint32_t j = 0; j < len[k]; ++j) s[j] = char(0x61 + wg_byte(ps, r * 32 + 16 + 5 * k + j / 8, j) % 26);
      x.sarr[k] = s;
    }
  }
}

// rp_list (xdrpp/rpcb_prot.x:24-37, the RPCBPROC_DUMP reply list): record
// r has k = 1 + draw(seed, r) % 4 nodes, k = WG_RP_LIST_LONG when
// r % 65536 == 65535.  Node g (its index over the whole batch, records in
// order): w0 = draw(ps, 8g), w1 = draw(ps, 8g + 1); r_prog = 100000 +
// w0 % 1000, r_vers = (w0 >> 32) % 5; |r_netid| = w1 % 9, |r_addr| =
// (w1 >> 16) % 25, |r_owner| = (w1 >> 32) % 13; byte j of r_netid from
// payload word 8g + 2 + j/8, r_addr 8g + 3 + j/8, r_owner 8g + 6 + j/8.
[[maybe_unused]] static uint32_t rp_list_nodes(uint64_t seed, uint64_t r) {
  return (r % 65536u == 65535u) ? WG_RP_LIST_LONG : 1u + uint32_t(wg_draw(seed, r) % 4u);
}
[[maybe_unused]] static void gen_rp_list(size_t n, uint64_t seed, vector<xdr::rp__list> &v) {
  v.clear();
  v.resize(n);
  const uint64_t ps = seed ^ WG_PAYLOAD_XOR;
  uint64_t g = 0;
  auto str = [&](xdr::xstring<> &s, uint32_t len, uint64_t w0) {
    string t(len, '\0');
    for (uint32_t j = 0; j < len; ++j) t[j] = char(wg_byte(ps, w0 + j / 8, j));
    s = t;
  };
  for (size_t r = 0; r < n; ++r) {
    const uint32_t k = rp_list_nodes(seed, r);
    xdr::rp__list *cur = &v[r];
    for (uint32_t i = 0; i < k; ++i, ++g) {
      if (i) {
        cur->rpcb_next.activate();
        cur = cur->rpcb_next.get();
      }
      const uint64_t w0 = wg_draw(ps, 8 * g), w1 = wg_draw(ps, 8 * g + 1);
      xdr::rpcb &m = cur->rpcb_map;
      m.r_prog = 100000u + uint32_t(w0 % 1000u);
      m.r_vers = uint32_t((w0 >> 32) % 5u);
      str(m.r_netid, uint32_t(w1 % 9u), 8 * g + 2);
      str(m.r_addr, uint32_t((w1 >> 16) % 25u), 8 * g + 3);
      str(m.r_owner, uint32_t((w1 >> 32) % 13u), 8 * g + 6);
    }
  }
}

[[maybe_unused]] static void fill_auth(xdr::opaque_auth &a, int32_t flavor, uint32_t len, uint64_t ps,
                      uint64_t word0) {
  a.flavor = xdr::auth_flavor(flavor);
  a.body.resize(len);
  for (uint32_t j = 0; j < len; ++j) a.body[j] = wg_byte(ps, word0 + j / 8, j);
}

[[maybe_unused]] static void gen_rpc(size_t n, uint64_t seed, vector<xdr::rpc_msg> &v) {
  v.resize(n);
  const uint64_t ps = seed ^ WG_PAYLOAD_XOR;
  for (size_t r = 0; r < n; ++r) {
    uint64_t d[16];
    for (int k = 0; k < 16; ++k) d[k] = wg_draw(seed, r * 16 + k);
    xdr::rpc_msg &m = v[r];
    m = xdr::rpc_msg{};
    m.xid = (uint32_t)d[0];
    unsigned sel = d[1] % 10;
    if (sel <= WG_RPC_CALL_MAX) {
      m.body.mtype(xdr::CALL);
      xdr::call_body &c = m.body.cbody();
      c.rpcvers = 2;
      c.prog = (uint32_t)d[2];
      c.vers = (uint32_t)d[3];
      c.proc = (uint32_t)d[4];
      fill_auth(c.cred, int32_t(d[5] % 2), d[6] % 401, ps, r * 128);
      fill_auth(c.verf, int32_t(d[7] % 2), d[8] % 401, ps, r * 128 + 64);
    } else {
      m.body.mtype(xdr::REPLY);
      xdr::reply_body &b = m.body.rbody();
      if (sel <= WG_RPC_PROG_UNAVAIL) {
        b.stat(xdr::MSG_ACCEPTED);
        fill_auth(b.areply().verf, int32_t(d[5] % 2), d[6] % 41, ps, r * 128 + 64);
        auto &rd = b.areply().reply_data;
        if (sel == WG_RPC_SUCCESS) rd.stat(xdr::SUCCESS);
        else if (sel == WG_RPC_PROG_MISMATCH) {
          rd.stat(xdr::PROG_MISMATCH);
          rd.mismatch_info().low = (uint32_t)d[9];
          rd.mismatch_info().high = (uint32_t)d[10];
        } else rd.stat(xdr::PROG_UNAVAIL);
      } else {
        b.stat(xdr::MSG_DENIED);
        if (sel == WG_RPC_RPC_MISMATCH) {
          b.rreply().stat(xdr::RPC_MISMATCH);
          b.rreply().mismatch_info().low = (uint32_t)d[9];
          b.rreply().mismatch_info().high = (uint32_t)d[10];
        } else {
          b.rreply().stat(xdr::AUTH_ERROR);
          b.rreply().rj_why() = xdr::auth_stat(d[11] % 15);
        }
      }
    }
  }
}

// ------------------------------------------------------------- staging
// Heap packing for encode inputs: payloads in record order, field order,
// no alignment (exercises unaligned heap reads on the device).
struct heap_t {
  vector<uint8_t> b;
  xdrg_bytes_ref put(const uint8_t *p, size_t n) {
    xdrg_bytes_ref r{b.size(), uint32_t(n), 0};
    b.insert(b.end(), p, p + n);
    return r;
  }
  // element array of a vector / pointer: 8-byte aligned, count elements
  xdrg_bytes_ref put_elems(const void *p, size_t count, size_t stride) {
    b.resize((b.size() + 7) & ~size_t(7), 0);
    xdrg_bytes_ref r{b.size(), uint32_t(count), 0};
    const uint8_t *q = static_cast<const uint8_t *>(p);
    b.insert(b.end(), q, q + count * stride);
    return r;
  }
};

[[maybe_unused]] static void stage(const vector<testns::numerics> &v, vector<uint8_t> &nat, heap_t &) {
  nat.resize(v.size() * sizeof(testns::numerics));
  memcpy(nat.data(), v.data(), nat.size());
}
[[maybe_unused]] static void stage(const vector<rec128> &v, vector<uint8_t> &nat, heap_t &) {
  nat.resize(v.size() * sizeof(rec128));
  memcpy(nat.data(), v.data(), nat.size());
}
[[maybe_unused]] static void stage(const vector<recvar> &v, vector<uint8_t> &nat, heap_t &h) {
  nat.assign(v.size() * sizeof(st_recvar), 0);
  st_recvar *s = reinterpret_cast<st_recvar *>(nat.data());
  for (size_t r = 0; r < v.size(); ++r) {
    s[r].id = v[r].id;
    s[r].kind = v[r].kind;
    s[r].blob = h.put(v[r].blob.data(), v[r].blob.size());
    s[r].name = h.put(reinterpret_cast<const uint8_t *>(v[r].name.data()), v[r].name.size());
    s[r].score = v[r].score;
  }
}
[[maybe_unused]] static void stage_auth(const xdr::opaque_auth &a, st_opaque_auth &s, heap_t &h) {
  s.flavor = a.flavor;
  s.body = h.put(a.body.data(), a.body.size());
}
[[maybe_unused]] static void stage(const vector<xdr::rpc_msg> &v, vector<uint8_t> &nat, heap_t &h) {
  nat.assign(v.size() * sizeof(st_rpc_msg), 0);
  st_rpc_msg *s = reinterpret_cast<st_rpc_msg *>(nat.data());
  for (size_t r = 0; r < v.size(); ++r) {
    const xdr::rpc_msg &m = v[r];
    s[r].xid = m.xid;
    s[r].body.mtype = m.body.mtype();
    if (m.body.mtype() == xdr::CALL) {
      const xdr::call_body &mc = m.body.cbody();
      st_call_body &c = s[r].body.u.cbody;
      c.rpcvers = mc.rpcvers;
      c.prog = mc.prog;
      c.vers = mc.vers;
      c.proc = mc.proc;
      stage_auth(mc.cred, c.cred, h);
      stage_auth(mc.verf, c.verf, h);
    } else {
      const xdr::reply_body &mb = m.body.rbody();
      st_reply_body &b = s[r].body.u.rbody;
      b.stat = mb.stat();
      if (mb.stat() == xdr::MSG_ACCEPTED) {
        const xdr::accepted_reply &a = mb.areply();
        stage_auth(a.verf, b.u.areply.verf, h);
        b.u.areply.reply_data.stat = a.reply_data.stat();
        if (a.reply_data.stat() == xdr::PROG_MISMATCH) {
          b.u.areply.reply_data.u.mismatch_info.low = a.reply_data.mismatch_info().low;
          b.u.areply.reply_data.u.mismatch_info.high = a.reply_data.mismatch_info().high;
        }
      } else {
        const xdr::rejected_reply &j = mb.rreply();
        b.u.rreply.stat = j.stat();
        if (j.stat() == xdr::RPC_MISMATCH) {
          b.u.rreply.u.mismatch_info.low = j.mismatch_info().low;
          b.u.rreply.u.mismatch_info.high = j.mismatch_info().high;
        } else
          b.u.rreply.u.rj_why = j.rj_why();
      }
    }
  }
}

[[maybe_unused]] static void stage(const vector<vecrec> &v, vector<uint8_t> &nat, heap_t &h) {
  nat.assign(v.size() * sizeof(st_vecrec), 0);
  st_vecrec *s = reinterpret_cast<st_vecrec *>(nat.data());
  for (size_t r = 0; r < v.size(); ++r) {
    const vecrec &x = v[r];
    s[r].id = x.id;
    s[r].vals = h.put_elems(x.vals.data(), x.vals.size(), 4);
    st_mismatch m{};
    if (x.opt) m = st_mismatch{x.opt->low, x.opt->high};
    s[r].opt = h.put_elems(&m, x.opt ? 1 : 0, sizeof m);
    vector<st_vpair> pv(x.pairs.size());
    for (size_t j = 0; j < pv.size(); ++j) {
      pv[j] = st_vpair{};
      pv[j].h = x.pairs[j].h;
      pv[j].b = x.pairs[j].b;
    }
    s[r].pairs = h.put_elems(pv.data(), pv.size(), sizeof(st_vpair));
    s[r].flag = x.flag;
  }
}

// containertest: {uvec ref, sarr[2] refs}; per record the element array
// (24-byte u_4_12: which, the arm at +8) then the two strings
struct st_u_4_12 {
  int32_t which;
  uint32_t pad;
  int32_t i;
  uint32_t pad2;
  double d;  // the f12 arm's double (0 for f4)
};
static_assert(sizeof(st_u_4_12) == 24, "u_4_12 staged element");
struct st_containertest {
  xdrg_bytes_ref uvec, sarr[2];
};
[[maybe_unused]] static void stage(const vector<testns::containertest> &v, vector<uint8_t> &nat, heap_t &h) {
  nat.assign(v.size() * sizeof(st_containertest), 0);
  st_containertest *s = reinterpret_cast<st_containertest *>(nat.data());
  for (size_t r = 0; r < v.size(); ++r) {
    const testns::containertest &x = v[r];
    vector<st_u_4_12> e(x.uvec.size());
    for (size_t j = 0; j < e.size(); ++j) {
      e[j] = st_u_4_12{};
      e[j].which = x.uvec[j].which();
      if (e[j].which == 12) {
        e[j].i = x.uvec[j].f12().i;
        e[j].d = x.uvec[j].f12().d;
      } else {
        e[j].i = x.uvec[j].f4().i;
      }
    }
    s[r].uvec = h.put_elems(e.data(), e.size(), sizeof(st_u_4_12));
    for (int k = 0; k < 2; ++k)
      s[r].sarr[k] = h.put(reinterpret_cast<const uint8_t *>(x.sarr[k].data()), x.sarr[k].size());
  }
}

// rp_list: per record (from an 8-byte boundary) the three strings of every
// node in node order, then, for k > 1 nodes, the images of nodes 1..k-1
// (8-byte aligned, contiguous); node i's rpcb_next = {image of node i + 1,
// 1}, the last node's {0, 0}.  Node 0's image is the record.
[[maybe_unused]] static void stage(const vector<xdr::rp__list> &v, vector<uint8_t> &nat, heap_t &h) {
  nat.assign(v.size() * sizeof(st_rp_list), 0);
  st_rp_list *s = reinterpret_cast<st_rp_list *>(nat.data());
  vector<st_rp_list> img;
  for (size_t r = 0; r < v.size(); ++r) {
    h.b.resize((h.b.size() + 7) & ~size_t(7), 0);
    img.clear();
    for (const xdr::rp__list *c = &v[r]; c; c = c->rpcb_next.get()) {
      st_rp_list e{};
      const xdr::rpcb &m = c->rpcb_map;
      e.rpcb_map.r_prog = m.r_prog;
      e.rpcb_map.r_vers = m.r_vers;
      e.rpcb_map.r_netid = h.put(reinterpret_cast<const uint8_t *>(m.r_netid.data()), m.r_netid.size());
      e.rpcb_map.r_addr = h.put(reinterpret_cast<const uint8_t *>(m.r_addr.data()), m.r_addr.size());
      e.rpcb_map.r_owner = h.put(reinterpret_cast<const uint8_t *>(m.r_owner.data()), m.r_owner.size());
      img.push_back(e);
    }
    if (img.size() > 1) {
      h.b.resize((h.b.size() + 7) & ~size_t(7), 0);
      const uint64_t base = h.b.size();
      for (size_t i = 0; i + 1 < img.size(); ++i) img[i].rpcb_next = xdrg_bytes_ref{base + 72 * i, 1, 0};
      h.b.insert(h.b.end(), reinterpret_cast<const uint8_t *>(img.data() + 1),
                 reinterpret_cast<const uint8_t *>(img.data() + img.size()));
    }
    s[r] = img[0];
  }
}

// Equality for round-trip checks (byte-level for fixed structs).
[[maybe_unused]] static bool same(const testns::numerics &a, const testns::numerics &b) {
  return a.b == b.b && a.i1 == b.i1 && a.i2 == b.i2 && a.i3 == b.i3 && a.i4 == b.i4 &&
         !memcmp(&a.f1, &b.f1, 4) && !memcmp(&a.f2, &b.f2, 8) && a.e1 == b.e1;
}
[[maybe_unused]] static bool same(const rec128 &a, const rec128 &b) { return !memcmp(&a, &b, sizeof a); }
[[maybe_unused]] static bool same(const recvar &a, const recvar &b) {
  return a.id == b.id && a.kind == b.kind && a.blob == b.blob && a.name == b.name &&
         !memcmp(&a.score, &b.score, 8);
}
[[maybe_unused]] static bool same(const vecrec &a, const vecrec &b) {
  return xdr::xdr_to_opaque(a) == xdr::xdr_to_opaque(b);
}
[[maybe_unused]] static bool same(const testns::containertest &a, const testns::containertest &b) {
  return xdr::xdr_to_opaque(a) == xdr::xdr_to_opaque(b);
}
[[maybe_unused]] static bool same(const xdr::rp__list &a, const xdr::rp__list &b) {
  return xdr::xdr_to_opaque(a) == xdr::xdr_to_opaque(b);
}
[[maybe_unused]] static bool same(const xdr::rpc_msg &a, const xdr::rpc_msg &b) {
  return xdr::xdr_to_opaque(a) == xdr::xdr_to_opaque(b);
}

}  // namespace refobj
#endif
