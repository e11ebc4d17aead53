/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Deterministic synthetic workloads for the four benchmark schemas
 * (SURVEY.md §8(d) configs 1-5).  The same specification is implemented in
 * numpy by xdrpp_amd/workloads.py; tests pin the two against each other
 * through the committed fixtures (tests/golden/manifest.json carries
 * sha256 of the full-size native inputs as well as the XDR outputs).
 *
 *   draw(seed, i) = splitmix64 finaliser of (seed + (i + 1) * GAMMA),
 *                   i.e. the i-th output of a splitmix64 stream.
 *
 * Staged native layouts (the device-side record representation) are the C
 * structs below; var-length bytes are xdrg_bytes_ref into a heap.
 */
#ifndef XDRG_WORKLOAD_GEN_H
#define XDRG_WORKLOAD_GEN_H
#include <stdint.h>
#include <string.h>
#include "../include/xdrgpu.h"

#define WG_GAMMA 0x9E3779B97F4A7C15ULL
#define WG_SEED_NUMERICS 0x5EED0001ULL
#define WG_SEED_REC128 0x5EED0002ULL
#define WG_SEED_RECVAR 0x5EED0003ULL
#define WG_SEED_RPC 0x5EED0004ULL
#define WG_SEED_REC128_MGPU 0x5EED0005ULL
#define WG_SEED_VECREC 0x5EED0006ULL
#define WG_SEED_CONTAINERTEST 0x5EED0008ULL
#define WG_SEED_RP_LIST 0x5EED0009ULL
#define WG_RP_LIST_LONG 500u       /* nodes of every 65536th list */
#define WG_PAYLOAD_XOR 0xB10BB10BB10BB10BULL

static inline uint64_t wg_draw(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * WG_GAMMA;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static inline uint8_t wg_byte(uint64_t seed, uint64_t word, uint32_t j) {
  return (uint8_t)(wg_draw(seed, word) >> (8 * (j & 7)));
}

/* ---- staged layouts ---------------------------------------------------- */
typedef struct {
  uint64_t id;
  int32_t kind;
  uint32_t pad_;
  xdrg_bytes_ref blob;
  xdrg_bytes_ref name;
  double score;
} st_recvar; /* 56 bytes */

typedef struct { int32_t flavor; uint32_t pad_; xdrg_bytes_ref body; } st_opaque_auth;
typedef struct { uint32_t low, high; } st_mismatch;
typedef struct { uint32_t rpcvers, prog, vers, proc; st_opaque_auth cred, verf; } st_call_body;
typedef struct { int32_t stat; union { st_mismatch mismatch_info; } u; } st_reply_data;
typedef struct { st_opaque_auth verf; st_reply_data reply_data; } st_accepted_reply;
typedef struct { int32_t stat; union { st_mismatch mismatch_info; int32_t rj_why; } u; } st_rejected_reply;
typedef struct { int32_t stat; uint32_t pad_; union { st_accepted_reply areply; st_rejected_reply rreply; } u; } st_reply_body;
typedef struct { int32_t mtype; uint32_t pad_; union { st_call_body cbody; st_reply_body rbody; } u; } st_body;
typedef struct { uint32_t xid; uint32_t pad_; st_body body; } st_rpc_msg; /* 80 bytes */

/* vecrec: element arrays live in the heap, each 8-byte aligned */
typedef struct { int64_t h; uint8_t b; uint8_t pad_[7]; } st_vpair; /* 16 bytes */
typedef struct {
  uint32_t id;
  uint32_t pad_;
  xdrg_bytes_ref vals;  /* int32[count] */
  xdrg_bytes_ref opt;   /* st_mismatch[0 or 1] */
  xdrg_bytes_ref pairs; /* st_vpair[count] */
  uint8_t flag;
  uint8_t pad2_[7];
} st_vecrec; /* 64 bytes */

/* rp_list (xdrpp/rpcb_prot.x:24-37): each node's image is the record's
 * layout; rpcb_next points at the next node's image in the heap */
typedef struct {
  uint32_t r_prog, r_vers;
  xdrg_bytes_ref r_netid, r_addr, r_owner;
} st_rpcb; /* 56 bytes */
typedef struct {
  st_rpcb rpcb_map;
  xdrg_bytes_ref rpcb_next; /* st_rp_list[0 or 1] */
} st_rp_list; /* 72 bytes */

/* rpc record kinds drawn per record: sel = draw1 % 10 */
enum { WG_RPC_CALL_MAX = 4, WG_RPC_SUCCESS = 5, WG_RPC_PROG_MISMATCH = 6,
       WG_RPC_PROG_UNAVAIL = 7, WG_RPC_RPC_MISMATCH = 8, WG_RPC_AUTH_ERROR = 9 };

#endif
