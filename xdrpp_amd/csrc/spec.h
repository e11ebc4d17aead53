// Plan-specialized kernels: source generation
// (codegen.cpp) and the code objects a plan carries (spec.cpp).
#pragma once
#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

struct xdrg_plan;

namespace xdrg {

constexpr int kSpecDevices = 64;

// Interface version of the generated kernels (their parameter lists and
// LDS layout, var_kernels.h): the source defines xdrg_spec_iface with it,
// and a code object that carries another value is refused at load.
constexpr unsigned kSpecIface = 15;

// The generated source of a plan and the launch facts it fixes.
struct spec_info {
  std::string source;     // HIP source over var_kernels.h
  uint32_t slots = 1;     // chunk-map slots per record the encode kernel uses
  uint64_t max_chunks = 0;  // 16-byte chunks those slots hold per record (bounds)
  bool dec_regs = false;  // the decode walks into registers: no native tile in LDS
  bool word_list = false; // the encode walks once into a word list (no walk per window)
  uint32_t list_words = 0; // ... of this many words per record (the mark included)
  uint64_t src_hash = 0;  // FNV-1a of the source (before the line that defines it)
  bool frame_walk = false;  // a recursive plan: the module holds the frame walks only
  bool tail_rx = false;     // ... and, a linked list (codegen.cpp tail_list), the index's record parse
};

// Kernels of one plan on one device.
struct spec_module {
  void *module = nullptr;  // hipModule_t
  void *f_size = nullptr, *f_enc = nullptr, *f_dec = nullptr, *f_dec_copy = nullptr;  // hipFunction_t
  void *f_ix_seg = nullptr;  // record-start parse of the plain-stream index (list ranking)
  void *f_rxs_walk = nullptr;  // ... and its speculative chain walk
  void *f_rxs_walk_whole = nullptr, *f_rxs_fix = nullptr;  // ... over records of any length
  void *f_enc_lb = nullptr, *f_enc_pre = nullptr;  // word-list plans: encode walked first (look-back / sized)
  // recursive plans: the frame walks (sub_kernels.h) over the plan's ops
  void *f_sub_size = nullptr, *f_sub_depth = nullptr, *f_sub_enc = nullptr, *f_sub_dec = nullptr;
  void *f_sub_chain = nullptr;  // the node pass (sub_kernels.h "Chains")
  void *f_sub_chain_size = nullptr;  // the size walk's chain pass (sub_kernels.h "Chains")
};

// A plan's specialized kernels: state 0 = not built yet, 1 = code object
// ready, -1 = unavailable (plan shape not generated, or the compile
// failed: the interpreter serves the plan).
struct spec_state {
  std::mutex mu;
  std::atomic<int> state{0};
  spec_info info;
  std::vector<char> code;  // gfx950 code object (ELF)
  std::string log;         // compile log of a failed build
  std::atomic<bool> loaded[kSpecDevices] = {};
  std::atomic<bool> failed[kSpecDevices] = {};  // the module did not load there: interpreter
  spec_module dev[kSpecDevices];
};

// Generate the specialized source of a var plan; false if the plan's shape
// is not handled (the interpreter runs it).
bool spec_source(const xdrg_plan &p, spec_info &info);

// Build (or find in the kernel cache) the plan's code object: 1 ready,
// -1 the plan runs on the interpreter.
int spec_build(const xdrg_plan &p);

// Ensure the plan's code object exists (cache, or hiprtc), then its module
// on the current device.  Returns the module, or nullptr when the plan runs
// on the interpreter.
const spec_module *spec_get(const xdrg_plan &p);

// Release the plan's modules (every device).
void spec_release(spec_state &s);

}  // namespace xdrg
