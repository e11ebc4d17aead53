// Plan-specialized kernels at plan time: the source codegen.cpp emits is
// compiled for gfx950 with hiprtc (the runtime form of an xdrc back end,
// SURVEY.md §8 f3) and loaded as a module on each device that launches the
// plan.  Code objects are cached on disk by a hash of their source, so a
// plan is compiled once per machine (or ahead of time, by build(), into the
// tree's kernel_cache/ that travels with it); a code object can also be
// attached directly (xdrg_plan_load_kernels).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

#include "plan.h"
#include "spec.h"

namespace xdrg {
namespace {

// The device headers the generated source includes, embedded at build
// time (build.py writes _embed.inc from dev_common.h, var_kernels.h and
// include/xdrgpu.h).
#include "_embed.inc"

const char *kOptsBase[] = {"-O3", "-std=c++17"};

// --offload-arch of the current device (gcnArchName without its feature
// suffix); gfx950 when the device cannot be asked.
std::string device_arch() {
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) {
    std::string a = prop.gcnArchName;
    const size_t k = a.find(':');
    if (k != std::string::npos) a.resize(k);
    if (!a.empty()) return a;
  }
  return "gfx950";
}

uint64_t fnv1a(const std::string &s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

// $XDRG_KERNEL_CACHE, else kernel_cache/ beside libxdrgpu.so; empty (no
// cache) when neither is known -- never a shared directory such as /tmp,
// where another user's file would be loaded as this plan's kernels.
std::string cache_dir() {
  if (const char *e = getenv("XDRG_KERNEL_CACHE")) return e;
  Dl_info di;
  if (dladdr(reinterpret_cast<void *>(&cache_dir), &di) && di.dli_fname) {
    std::string so = di.dli_fname;
    const size_t k = so.rfind('/');
    return (k == std::string::npos ? std::string(".") : so.substr(0, k)) + "/kernel_cache";
  }
  return "";
}

std::string cache_key(const std::string &src, const std::string &arch) {
  uint64_t h = fnv1a(src);
  for (const char *hd : kEmbedText) h = fnv1a(hd, h);
  for (const char *o : kOptsBase) h = fnv1a(o, h);
  h = fnv1a(arch, h);
  char b[32];
  snprintf(b, sizeof b, "%016llx", static_cast<unsigned long long>(h));
  return b;
}

bool read_file(const std::string &path, std::vector<char> &out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return !out.empty();
}

void write_file(const std::string &path, const char *data, size_t n) {
  const std::string tmp = path + ".tmp" + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    if (!f) return;
    f.write(data, static_cast<std::streamsize>(n));
    if (!f) return;
  }
  std::rename(tmp.c_str(), path.c_str());  // atomic on one file system
}

// hiprtc: source -> gfx950 code object.
bool rtc_compile(const std::string &src, const std::string &arch, std::vector<char> &code, std::string &log) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "xdrg_spec.hip", kEmbedCount, kEmbedText, kEmbedName) !=
      HIPRTC_SUCCESS) {
    log = "hiprtcCreateProgram failed";
    return false;
  }
  const std::string oa = "--offload-arch=" + arch;
  const char *opts[] = {oa.c_str(), kOptsBase[0], kOptsBase[1]};
  const hiprtcResult rc = hiprtcCompileProgram(prog, sizeof opts / sizeof opts[0], opts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  log.assign(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &log[0]);
  bool ok = rc == HIPRTC_SUCCESS;
  if (ok) {
    size_t cs = 0;
    ok = hiprtcGetCodeSize(prog, &cs) == HIPRTC_SUCCESS && cs > 0;
    if (ok) {
      code.resize(cs);
      ok = hiprtcGetCode(prog, code.data()) == HIPRTC_SUCCESS;
    }
  }
  hiprtcDestroyProgram(&prog);
  return ok;
}

}  // namespace

// Builds (or finds) the plan's code object; state 1 on success, -1 when the
// plan runs on the interpreter.
int spec_build(const xdrg_plan &cp) {
  xdrg_plan &p = const_cast<xdrg_plan &>(cp);
  spec_state &s = p.spec;
  const int st = s.state.load(std::memory_order_acquire);
  if (st != 0) return st;
  std::lock_guard<std::mutex> g(s.mu);
  if (s.state.load(std::memory_order_relaxed) != 0) return s.state.load();
  if (s.code.empty()) {
    if (!spec_source(p, s.info)) {
      s.state.store(-1, std::memory_order_release);
      return -1;
    }
    const std::string arch = device_arch(), dir = cache_dir(), key = cache_key(s.info.source, arch);
    const std::string co = dir + "/" + key + ".co";
    if (dir.empty() || !read_file(co, s.code)) {
      std::string log;
      if (!rtc_compile(s.info.source, arch, s.code, log)) {
        s.log = log;
        s.code.clear();
        s.state.store(-1, std::memory_order_release);
        return -1;
      }
      if (!dir.empty()) {
        mkdir(dir.c_str(), 0755);  // a read-only tree just means no cache
        write_file(co, s.code.data(), s.code.size());
        write_file(dir + "/" + key + ".hip", s.info.source.data(), s.info.source.size());
      }
    }
  }
  s.state.store(1, std::memory_order_release);
  return 1;
}

const spec_module *spec_get(const xdrg_plan &cp) {
  if (spec_build(cp) != 1) return nullptr;
  xdrg_plan &p = const_cast<xdrg_plan &>(cp);
  spec_state &s = p.spec;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kSpecDevices) return nullptr;
  if (s.loaded[dev].load(std::memory_order_acquire)) return &s.dev[dev];
  if (s.failed[dev].load(std::memory_order_acquire)) return nullptr;
  std::lock_guard<std::mutex> g(s.mu);
  if (s.loaded[dev].load(std::memory_order_relaxed)) return &s.dev[dev];
  if (s.failed[dev].load(std::memory_order_relaxed)) return nullptr;
  // a load that fails is not retried on every launch: the plan runs on the
  // interpreter on this device from now on
  auto fail = [&](hipModule_t m, const char *why) -> const spec_module * {
    if (m) (void)hipModuleUnload(m);
    s.log = why;
    s.failed[dev].store(true, std::memory_order_release);
    return nullptr;
  };
  hipModule_t m = nullptr;
  if (hipModuleLoadData(&m, s.code.data()) != hipSuccess)
    return fail(nullptr, "specialized kernels: the code object does not load on this device");
  spec_module &d = s.dev[dev];
  if (s.info.frame_walk) {  // a recursive plan: the frame walks only
    hipFunction_t g[6] = {};
    const char *gn[6] = {"xdrg_spec_sub_size", "xdrg_spec_sub_depth", "xdrg_spec_sub_encode", "xdrg_spec_sub_decode",
                         "xdrg_spec_sub_chain", "xdrg_spec_sub_chain_size"};
    for (int i = 0; i < 6; ++i)
      if (hipModuleGetFunction(&g[i], m, gn[i]) != hipSuccess)
        return fail(m, "specialized kernels: the code object lacks a frame walk");
    d.f_sub_size = g[0];
    d.f_sub_depth = g[1];
    d.f_sub_enc = g[2];
    d.f_sub_dec = g[3];
    d.f_sub_chain = g[4];
    d.f_sub_chain_size = g[5];
  }
  hipFunction_t f[8] = {};
  const char *names[8] = {"xdrg_spec_size",     "xdrg_spec_encode",         "xdrg_spec_decode",
                          "xdrg_spec_decode_copy", "xdrg_spec_ix_seg",      "xdrg_spec_rxs_walk",
                          "xdrg_spec_rxs_walk_whole", "xdrg_spec_rxs_fix"};
  for (int i = s.info.frame_walk ? 4 : 0; i < 8 && (!s.info.frame_walk || s.info.tail_rx); ++i)
    if (hipModuleGetFunction(&f[i], m, names[i]) != hipSuccess)
      return fail(m, "specialized kernels: the code object lacks a kernel");
  // a code object of another kernel interface (an older build's AOT file),
  // or of another plan's source (a foreign cache file or attached object,
  // whose hard-coded offsets would silently write wrong bytes)
  void *iv = nullptr;
  size_t ib = 0;
  unsigned iface = 0;
  if (hipModuleGetGlobal(&iv, &ib, m, "xdrg_spec_iface") != hipSuccess || ib != sizeof iface ||
      hipMemcpyDtoH(&iface, iv, sizeof iface) != hipSuccess || iface != kSpecIface)
    return fail(m, "specialized kernels: code object of another kernel interface (rebuild it from "
                   "xdrg_plan_kernel_source)");
  unsigned long long sh = 0;
  if (hipModuleGetGlobal(&iv, &ib, m, "xdrg_spec_src_hash") != hipSuccess || ib != sizeof sh ||
      hipMemcpyDtoH(&sh, iv, sizeof sh) != hipSuccess || sh != s.info.src_hash)
    return fail(m, "specialized kernels: code object compiled from another plan's source");
  d.module = m;
  d.f_size = f[0];
  d.f_enc = f[1];
  d.f_dec = f[2];
  d.f_dec_copy = f[3];
  d.f_ix_seg = f[4];
  d.f_rxs_walk = f[5];
  d.f_rxs_walk_whole = f[6];
  d.f_rxs_fix = f[7];
  if (s.info.word_list) {  // the walk-first encode, generated for word-list plans only
    hipFunction_t a = nullptr, b = nullptr;
    if (hipModuleGetFunction(&a, m, "xdrg_spec_encode_lb") != hipSuccess ||
        hipModuleGetFunction(&b, m, "xdrg_spec_encode_pre") != hipSuccess)
      return fail(m, "specialized kernels: the code object lacks the walk-first encode");
    d.f_enc_lb = a;
    d.f_enc_pre = b;
  }
  s.loaded[dev].store(true, std::memory_order_release);
  return &d;
}

void spec_release(spec_state &s) {
  int cur = 0;
  const bool restore = hipGetDevice(&cur) == hipSuccess;
  for (int d = 0; d < kSpecDevices; ++d)
    if (s.dev[d].module) {
      (void)hipSetDevice(d);
      (void)hipModuleUnload(static_cast<hipModule_t>(s.dev[d].module));
      s.dev[d].module = nullptr;
    }
  if (restore) (void)hipSetDevice(cur);
}

}  // namespace xdrg

extern "C" {

int xdrg_plan_kernel_source(const xdrg_plan *p, char *buf, size_t cap, size_t *len) {
  if (!p || !len) return XDRG_EINVAL;
  xdrg::spec_info info;
  if (!xdrg::spec_source(*p, info)) return XDRG_EUNSUPPORTED;
  *len = info.source.size();
  if (buf && cap) {
    const size_t k = std::min(cap - 1, info.source.size());
    std::memcpy(buf, info.source.data(), k);
    buf[k] = '\0';
  }
  return XDRG_OK;
}

int xdrg_plan_build_kernels(xdrg_plan *p) {
  if (!p) return XDRG_EINVAL;
  if (p->path != XDRG_PATH_VAR) return XDRG_EUNSUPPORTED;
  if (xdrg::spec_build(*p) == 1) return XDRG_OK;
  if (!p->spec.log.empty()) return xdrg::record_hip_error(hipErrorInvalidImage, p->spec.log.c_str());
  return XDRG_EUNSUPPORTED;
}

int xdrg_plan_load_kernels(xdrg_plan *p, const void *code, size_t size) {
  if (!p || !code || !size) return XDRG_EINVAL;
  if (p->path != XDRG_PATH_VAR) return XDRG_EUNSUPPORTED;
  std::lock_guard<std::mutex> g(p->spec.mu);
  if (p->spec.state.load() != 0) return XDRG_EINVAL;  // already built or in use
  if (!xdrg::spec_source(*p, p->spec.info)) return XDRG_EUNSUPPORTED;
  const char *c = static_cast<const char *>(code);
  p->spec.code.assign(c, c + size);
  return XDRG_OK;
}

}  // extern "C"
