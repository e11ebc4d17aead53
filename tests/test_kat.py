"""The known answers of SURVEY.md §8(c) and the past-bound encode of
§8(a) a4, from the REAL reference (oracle/ref_golden kat over the genuine
xdrc output of oracle/x/kat.x, tests/golden/kat.json):

  union u(RED) with int arm -1          -> 00000000ffffffff
  xvector<int>{1, 2}                    -> 00000002 00000001 00000002
  {-2, 0x0102..08, 1.5, blob{1,2,3}, "hello"}
                                        -> fffffffe 0102030405060708
                                           3ff8000000000000 00000003
                                           01020300 00000005 68656c6c 6f000000
  a 65-byte opaque<64> (9-char string<8>, 3-element int<2>) encodes
  without error (xdr_generic_put checks capacity only, marshal.h:118-127);
  its decode throws "xvector overflow" / "xstring overflow"
  (types.h:486-489, :539-542).

The union and the xvector are encoded as the one-field structs a plan
describes (the generator checks the bytes are the same as alone).  The
GPU runs every case through the plan-specialized kernels and the
interpreter.
"""
import os

import numpy as np
import pytest

from conftest import ROOT

from xdrpp_amd import objects as OB
from xdrpp_amd.xdr_types import (Double, Enum, Int, Opaque, String, Struct, UHyper, Union, Void,
                                 XVector, compile_plan)
import oracle_bridge as O

kcolor = Enum("kcolor", {"KRED": 0, "KREDDER": 1, "KREDDEST": 2})
ku = Union("ku", "c", kcolor, [([0], "i", Int), ([1], "h", UHyper)], default=("", Void))
ku_rec = Struct("ku_rec", [("u", ku)])
kint_vec = Struct("kint_vec", [("v", XVector(Int))])
kstruct = Struct("kstruct", [("i", Int), ("u", UHyper), ("d", Double), ("blob", Opaque(64)),
                             ("name", String())])
kbounded = Struct("kbounded", [("blob", Opaque(64)), ("s", String(8)), ("v", XVector(Int, 2))])
TYPES = {"ku_rec": ku_rec, "kint_vec": kint_vec, "kstruct": kstruct, "kbounded": kbounded}


def bounded(nb, ns, nv):
    return {"blob": bytes(range(1, nb + 1)), "s": bytes(ord("a") + j for j in range(ns)),
            "v": [10 + j for j in range(nv)]}


# (kat.json key, type, value)
VALUES = [
    ("union_red_m1", ku_rec, {"u": (0, -1)}),
    ("union_redder", ku_rec, {"u": (1, 0x0102030405060708)}),
    ("union_default", ku_rec, {"u": (2, None)}),
    ("xvector_int_1_2", kint_vec, {"v": [1, 2]}),
    ("struct_hello", kstruct, {"i": -2, "u": 0x0102030405060708, "d": 1.5, "blob": b"\x01\x02\x03",
                               "name": b"hello"}),
    ("bounded_in", kbounded, bounded(64, 8, 2)),
    ("bounded_over_all", kbounded, bounded(65, 9, 3)),
    ("bounded_over_blob", kbounded, bounded(65, 8, 2)),
    ("bounded_over_s", kbounded, bounded(64, 9, 2)),
    ("bounded_over_v", kbounded, bounded(64, 8, 3)),
]
ERRORS = ["kbounded_in", "kbounded_over_blob", "kbounded_over_s", "kbounded_over_v", "kbounded_over_all"]
SURVEY = {"union_red_m1": "00000000ffffffff", "xvector_int_1_2": "000000020000000100000002",
          "struct_hello": "fffffffe" "0102030405060708" "3ff8000000000000" "00000003" "01020300"
                          "00000005" "68656c6c" "6f000000"}


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("name", list(TYPES))
def test_descriptors_equal_kat_x(name):
    import xdrc_front as xdrc
    from test_xdrc import same_plan
    sp = xdrc.load_file(os.path.join(ROOT, "oracle", "x", "kat.x"))
    assert same_plan(sp.plan(name), compile_plan(TYPES[name]))


def test_survey_probes(kat):
    """The reference's bytes are the ones SURVEY §8(c) probed."""
    for k, v in SURVEY.items():
        assert kat[k] == v


@pytest.mark.parametrize("key,t,value", VALUES, ids=[v[0] for v in VALUES])
def test_oracle_known_answers(kat, key, t, value):
    cp = compile_plan(t)
    nat, heap = OB.stage(t, [value])
    x, _ = O.encode(cp, nat, 1, heap)
    assert bytes(x).hex() == kat[key]


EXC = {"none": 0, "xvector overflow": 3, "xstring overflow": 4}


@pytest.mark.parametrize("case", ERRORS)
def test_oracle_bound_errors(kat, case):
    c = kat["errors"][case]
    x = np.frombuffer(bytes.fromhex(c["input"]), dtype=np.uint8).copy()
    offs = np.array([0, x.size], dtype=np.uint64)
    try:
        O.decode(compile_plan(kbounded), x, 1, offs)
        code = 0
    except O.OracleError as e:
        code = e.code
    assert code == EXC[c["what"] or "none"]


# ------------------------------------------------------------------ GPU
PATHS = {"specialized": {"specialize": 1}, "interpreter": {"specialize": 0, "var_encode_kernel": 1,
                                                          "var_decode_kernel": 1},
         "interpreter_window": {"specialize": 0, "var_encode_kernel": 3, "var_decode_kernel": 2}}


@pytest.mark.gpu
@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("key,t,value", VALUES, ids=[v[0] for v in VALUES])
def test_gpu_known_answers(kat, dev, path, key, t, value):
    """Encode (a past-bound field encodes, as in the reference), then the
    decode of the reference's bytes: a round trip in bound, the reference's
    exception and what() past it."""
    import torch
    from xdrpp_amd import marshal as M
    mar = M.Marshaler(M.Plan(t, PATHS[path]), dev)
    nat, heap = OB.stage(t, [value])
    r = mar.encode(torch.from_numpy(nat).to(dev), 1, torch.from_numpy(heap).to(dev) if heap.size else None)
    assert r.xdr.cpu().numpy().tobytes().hex() == kat[key]
    x = torch.from_numpy(np.frombuffer(bytes.fromhex(kat[key]), dtype=np.uint8).copy()).to(dev)
    offs = torch.tensor([0, x.numel()], dtype=torch.int64, device=dev)
    err = kat["errors"].get("k" + key) if key.startswith("bounded") else None
    if err and err["exception"] != "none":
        with pytest.raises(M.XdrOverflow) as e:
            mar.decode(x, 1, offs)
        assert str(e.value) == err["what"] and e.value.record == 0
        return
    nat2, heap2 = mar.decode(x, 1, offs)
    assert OB.unstage(t, nat2.cpu().numpy(), heap2.cpu().numpy(), 1) == [value]
