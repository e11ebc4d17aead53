// ORACLE / TEST INFRASTRUCTURE ONLY.
//
// The reference types the oracle marshals, as GENUINE xdrc output: the
// reference's own back end (xdrc/gen_hh.cc, driven by oracle/xdrc_driver.cc
// over the AST oracle/xdrc_front.py builds; oracle/Makefile) run on
//   tests/xdrtest.x     -> tests/xdrtest.hh   numerics, the container types
//   xdrpp/rpc_msg.x     -> xdrpp/rpc_msg.hh   rpc_msg (also what server.h uses)
//   xdrpp/rpcb_prot.x   -> xdrpp/rpcb_prot.hh rp__list (the rp_list batch)
//   oracle/x/bench.x    -> bench.hh           rec128, recvar, vecrec
//   oracle/x/validated.x -> validated.hh      numerics in testns_v
//   oracle/x/kat.x      -> kat.hh             the SURVEY §8(c) known-answer types
// testns_v opts in to enum validation with the idiom of the reference's
// tests/validate.cc:18-20.
#ifndef XDRG_REF_TYPES_HH
#define XDRG_REF_TYPES_HH
#include <xdrpp/marshal.h>
#include <xdrpp/rpc_msg.hh>
#include <xdrpp/rpcb_prot.hh>

#include "bench.hh"
#include "kat.hh"
#include "tests/xdrtest.hh"
#include "validated.hh"

namespace testns_v {
template <typename T> inline void xdr_validate_enum(T);
}

static_assert(sizeof(rec128) == 128, "rec128 native layout");
#endif
