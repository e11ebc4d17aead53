// xdrc back end: device plans at generation time (gen_plan.cc).
//
// Compiled into xdrc beside gen_hh.cc (xdrc/gen_hh.cc:817-899), against
// xdrc's own AST (xdrc/xdrc_internal.h), and linked with libxdrgpu.so for
// the kernel sources (host-only calls).  `xdrc -plan file.x` writes the plan
// header; include it after the header `xdrc -hh file.x` writes (and after
// include/xdrpp_gpu.hh) to give xdr::gpu::plan_for<T>() the emitted plans.
//
// xdrc/xdrc_internal.h has no include guard: include it first, then this.
#pragma once
#include <iosfwd>
#include <set>
#include <string>
#include <vector>

namespace xdrg_gen {

struct plan_gen_options {
  std::string input;                    // the .x file's name (the header's comment)
  std::string guard;                    // the plan header's include guard
  std::string xdr_guard;                // the include guard of xdrc -hh's header for the same file
  std::set<std::string> validate_enums; // enums whose C++ type opts in to xdr_validate_enum
  std::string kernel_dir;               // "": no kernel sources; else <dir>/<type>.hip
  std::vector<std::string> kernel_types;  // types to write kernels for (empty: every variable-length one)
};

// Write the plan header of every struct and union of `syms`; 0, or 1 when a
// kernel source could not be written.
int gen_plan(std::ostream &os, const symlist_t &syms, const plan_gen_options &opt);

}  // namespace xdrg_gen
