"""Regenerate tests/golden/ from the REAL reference marshaler.

ORACLE / TEST INFRASTRUCTURE ONLY.  Needs oracle/_ref/ref_golden (built by
`make -C oracle` from /root/reference sources in place).  Writes

  tests/golden/<schema>_<n>.{native,heap,xdr,offsets}   small fixtures
  tests/golden/kat.json                                  known answers + error cases
  tests/golden/manifest.json                             sizes + sha256 of
                                                         full-size reference outputs

Full-size outputs (1M records) are hashed, not committed.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(ROOT, "tests", "golden")
BIN = os.path.join(HERE, "_ref", "ref_golden")

SMALL = {"numerics": 1000, "rec128": 1024, "recvar": 1024, "rpc": 1024, "vecrec": 1024, "containertest": 1024,
         "rp_list": 1024}
FULL = {"rec128": 1 << 20, "recvar": 1 << 20, "rpc": 1 << 20, "numerics": 1 << 16,
        "rec128_mgpu": 1 << 24}
FULL2 = {"numerics": 1 << 20}  # second full-size entries (dict keys are unique per schema)
MID = {"recvar": 1 << 16, "rpc": 1 << 16, "vecrec": 1 << 16, "containertest": 1 << 16, "rp_list": 1 << 16}
FULL3 = {"vecrec": 1 << 20, "containertest": 1 << 20, "rp_list": 1 << 20}
EXTS = ("native", "heap", "xdr", "offsets", "msgs", "msgoffs")
NOMSGS = {"rec128_mgpu"}  # 16M records: messages hashed only where they are tested


def sha(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


RPC_SMALL = 1024
RPC_FULL = 1 << 20


def rpc_fixtures(manifest: dict) -> None:
    """RPC header batches: the dispatch stream comes from
    xdrpp_amd.workloads.rpc_calls (inputs), the expected headers, client
    statuses and error replies from the reference (ref_golden rpc)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    from xdrpp_amd import workloads as W
    procs = os.path.join(GOLD, "rpc_procs.bin")
    W.RPC_PROCS.astype("<u4").tofile(procs)
    stream, offs = W.rpc_calls(RPC_SMALL)
    pre = os.path.join(GOLD, f"rpccall_{RPC_SMALL}")
    stream.tofile(pre + ".stream")
    offs.astype("<u8").tofile(pre + ".msgoffs")
    subprocess.check_call([BIN, "rpc", pre + ".stream", pre + ".msgoffs", procs, "-", pre])
    # client side over the config-4 messages: expected xid = the message's
    # own xid, every 7th one flipped
    msgs = np.fromfile(os.path.join(GOLD, f"rpc_{SMALL['rpc']}.msgs"), dtype=np.uint8)
    moff = np.fromfile(os.path.join(GOLD, f"rpc_{SMALL['rpc']}.msgoffs"), dtype="<u8")
    xids = msgs.view(">u4")[(moff[:-1] // 4 + 1).astype(np.int64)].astype("<u4")
    xids[::7] ^= 1
    cpre = os.path.join(GOLD, f"rpc_{SMALL['rpc']}")
    xids.tofile(cpre + ".xids")
    with tempfile.TemporaryDirectory() as td:
        subprocess.check_call([BIN, "rpc", cpre + ".msgs", cpre + ".msgoffs", procs,
                               cpre + ".xids", os.path.join(td, "c")])
        shutil.copy(os.path.join(td, "c.chk"), cpre + ".chk")
        stream, offs = W.rpc_calls(RPC_FULL)
        fp = os.path.join(td, "full")
        stream.tofile(fp + ".stream")
        offs.astype("<u8").tofile(fp + ".msgoffs")
        subprocess.check_call([BIN, "rpc", fp + ".stream", fp + ".msgoffs", procs, "-", fp])
        manifest["hashes"][f"rpccall_{RPC_FULL}"] = {
            "n": RPC_FULL, **{e: sha(fp + "." + e) for e in ("stream", "hdrs", "chk", "replies")},
            "stream_bytes": os.path.getsize(fp + ".stream")}


SUCCESS_N = 512


def success_fixtures() -> None:
    """Success replies xdr_to_msg(rpc_success_hdr(xid), res) of rec128
    results from the reference (ref_golden success; xdrpp/server.h:27-49,
    srpc.h:152), and rpc_success_hdr(7)'s message, which ref_golden checks
    equals rpc_msg(7, REPLY)'s as tests/arpc.cc:35-43 does."""
    subprocess.check_call([BIN, "success", str(SUCCESS_N), os.path.join(GOLD, f"success_rec128_{SUCCESS_N}")])


def depth_fixtures() -> None:
    """depth_checker (xdrpp/depth_checker.h): the smallest passing limit of
    every record of the small batches, from the real check_xdr_depth."""
    for schema, n in SMALL.items():
        subprocess.check_call([BIN, "depths", schema, str(n),
                               os.path.join(GOLD, f"{schema}_{n}.depths")])


def full_hashes(manifest: dict, entries) -> None:
    """sha256 of the reference's outputs for (schema, n) batches."""
    with tempfile.TemporaryDirectory() as td:
        for schema, n in entries:
            pre = os.path.join(td, f"{schema}_{n}")
            extra = ["nomsgs"] if schema in NOMSGS else []
            subprocess.check_call([BIN, "gen", schema, str(n), pre] + extra)
            exts = [e for e in EXTS if os.path.exists(pre + "." + e)]
            manifest["hashes"][f"{schema}_{n}"] = {
                "n": n, **{e: sha(pre + "." + e) for e in exts},
                "xdr_bytes": os.path.getsize(pre + ".xdr")}
            for e in exts:
                os.remove(pre + "." + e)


def main() -> int:
    if "--only-full" in sys.argv:  # --only-full schema:n [schema:n ...]
        mp = os.path.join(GOLD, "manifest.json")
        manifest = json.load(open(mp))
        i = sys.argv.index("--only-full")
        full_hashes(manifest, [(a.split(":")[0], int(a.split(":")[1])) for a in sys.argv[i + 1:]])
        with open(mp, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return 0
    if "--only-small" in sys.argv:  # --only-small schema [schema ...]: fixtures + depths of those
        mp = os.path.join(GOLD, "manifest.json")
        manifest = json.load(open(mp))
        for schema in sys.argv[sys.argv.index("--only-small") + 1:]:
            n = SMALL[schema]
            pre = os.path.join(GOLD, f"{schema}_{n}")
            subprocess.check_call([BIN, "gen", schema, str(n), pre])
            manifest["small"][schema] = {"n": n, "files": {e: f"{schema}_{n}.{e}" for e in EXTS},
                                         "xdr_bytes": os.path.getsize(pre + ".xdr")}
            subprocess.check_call([BIN, "depths", schema, str(n), pre + ".depths"])
        with open(mp, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return 0
    if "--only-success" in sys.argv:
        success_fixtures()
        return 0
    if "--only-depths" in sys.argv:
        depth_fixtures()
        return 0
    if "--only-rpc" in sys.argv:
        mp = os.path.join(GOLD, "manifest.json")
        manifest = json.load(open(mp))
        rpc_fixtures(manifest)
        with open(mp, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return 0
    if not os.path.exists(BIN):
        print("build oracle/_ref/ref_golden first (make -C oracle)", file=sys.stderr)
        return 2
    os.makedirs(GOLD, exist_ok=True)
    manifest = {"generator": "oracle/ref_golden.cc (reference xdrpp/marshal.cc + server side compiled in place, genuine xdrc-generated types)",
                "small": {}, "hashes": {}}
    for schema, n in SMALL.items():
        pre = os.path.join(GOLD, f"{schema}_{n}")
        subprocess.check_call([BIN, "gen", schema, str(n), pre])
        manifest["small"][schema] = {"n": n, "files": {e: f"{schema}_{n}.{e}" for e in EXTS},
                                     "xdr_bytes": os.path.getsize(pre + ".xdr")}
    subprocess.check_call([BIN, "kat", os.path.join(GOLD, "kat.json")])
    full_hashes(manifest, [kv for table in (FULL, FULL2, MID, FULL3) for kv in table.items()])
    rpc_fixtures(manifest)
    success_fixtures()
    depth_fixtures()
    with open(os.path.join(GOLD, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", GOLD)
    return 0


if __name__ == "__main__":
    sys.exit(main())
