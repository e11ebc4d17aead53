"""Framing of record-marked messages of any length (xdrg_index_msgs with
max_msg_len past one index window).

read_message (xdrpp/srpc.cc:29-55) frames messages of any size; msg_sock
(msgsock.cc:97-111) rejects those above its maxmsglen, 1 MiB by default
(msgsock.h:29).  The device index keeps its list-ranking windows for
messages up to XDRG_INDEX_MAX_MSG and walks longer ones mark by mark
(xdrpp_amd/csrc/xdrgpu.hip ix_windows).

Golden framing: tests/golden/frames.json, the REAL read_message over the
seeded streams of tests/msg_streams.py (oracle/ref_golden frame; script
tests/golden/make_frames.py).  Streams mix 0-byte to 1 MiB messages.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from conftest import GOLD

from xdrpp_amd import _abi as A
import msg_streams as MS
import oracle_bridge as O

REF = "/root/reference"
WHAT = {None: 0, "too long": A.ERR_MSG_TOO_LONG, "read_message: premature EOF": A.ERR_MSG_EOF,
        "read_message: message fragments unimplemented": A.ERR_MSG_FRAGMENT,
        "read_message: received size not multiple of 4": A.ERR_MSG_SIZE4}


@pytest.fixture(scope="module")
def frames():
    with open(os.path.join(GOLD, "frames.json")) as f:
        return json.load(f)


_streams = {}


def stream(name):
    if name not in _streams:
        _streams[name] = MS.stream(name)
    return _streams[name]


def want_of(r):
    """(error code, count, offsets[:count+1]) of a fixture framing."""
    offs = np.array(r["offsets"], dtype=np.uint64)
    return WHAT[r["what"]], offs.size - 1, offs


# ------------------------------------------------------------------ CPU
def test_streams_regenerate(frames):
    for name, st in frames["streams"].items():
        x = stream(name)
        assert (x.size, MS.sha256(x)) == (st["bytes"], st["sha256"]), name


@pytest.mark.parametrize("i", range(len(MS.FRAMINGS)))
def test_oracle_framing(frames, i):
    """The C restatement frames as the reference does, at any length."""
    r = frames["framings"][i]
    code, cnt, offs = want_of(r)
    rc, ocnt, ooffs = O.index_msgs(stream(r["stream"]), r["max_msg_len"])
    assert (rc, ocnt) == (code, cnt)
    assert np.array_equal(ooffs, offs)


def test_workspace_size():
    L = A.lib()
    assert L.xdrg_index_workspace_size(1 << 20, A.MSG_SOCK_MAXMSGLEN) > L.xdrg_index_workspace_size(1 << 20, 16380)
    assert L.xdrg_index_workspace_size(1 << 20, A.MAX_MSG) > 0


@pytest.mark.skipif(not os.path.exists(f"{REF}/xdrpp/srpc.cc"), reason="reference tree absent")
def test_fixture_regenerates(tmp_path):
    import subprocess
    import sys
    before = open(os.path.join(GOLD, "frames.json"), "rb").read()
    subprocess.run([sys.executable, os.path.join(GOLD, "make_frames.py")], check=True)
    assert open(os.path.join(GOLD, "frames.json"), "rb").read() == before


# ------------------------------------------------------------------ GPU
def device_index(x, dev, maxlen, max_msgs=None):
    """(error code, count, offsets[:count+1]) of xdrg_index_msgs: the
    offsets up to the failing mark on an error, as the oracle gives them."""
    import torch
    from xdrpp_amd import marshal as M
    L = A.lib()
    if max_msgs is None:
        max_msgs = x.size // 4
    t = torch.from_numpy(x).to(dev) if x.size else torch.empty(0, dtype=torch.uint8, device=dev)
    ws = torch.empty(max(L.xdrg_index_workspace_size(x.size, maxlen), 16), dtype=torch.uint8, device=dev)
    offs = torch.empty(max_msgs + 1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    st = M.Status(dev)
    s = torch.cuda.current_stream().cuda_stream
    st.init(s)
    A.check(L.xdrg_index_msgs(C.c_void_p(t.data_ptr() if x.size else None), x.size, maxlen, max_msgs,
                              C.c_void_p(offs.data_ptr()), C.c_void_p(cnt.data_ptr()),
                              C.c_void_p(ws.data_ptr()), ws.numel(), st.ptr, s), "xdrg_index_msgs")
    e = st.read(s)
    n = int(e.record) if e.code else int(cnt.item())
    return int(e.code), n, offs[:n + 1].cpu().numpy().view(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(len(MS.FRAMINGS)))
def test_gpu_framing(frames, dev, i):
    """8-byte to 1 MiB messages framed on the device exactly as read_message
    frames them; MSG_TOO_LONG only above the caller's max_msg_len."""
    r = frames["framings"][i]
    code, cnt, offs = want_of(r)
    got = device_index(stream(r["stream"]), dev, r["max_msg_len"])
    assert got[:2] == (code, cnt)
    assert np.array_equal(got[2], offs)


@pytest.mark.gpu
@pytest.mark.parametrize("max_msgs", [0, 1, 5, 25, 39, 40])
def test_gpu_capacity(dev, max_msgs):
    """The index's capacity (max_msgs) among long messages: MSG_COUNT at
    the first message past it, as the oracle."""
    x = stream("mixed")
    want = O.index_msgs(x, MS.MIB, max_msgs)
    got = device_index(x, dev, MS.MIB, max_msgs)
    assert got[:2] == want[:2]
    assert np.array_equal(got[2], want[2])


@pytest.mark.gpu
def test_gpu_windows_vs_oracle_fuzzed(dev):
    """Damaged long-message streams (flipped bytes, words that read as
    marks) against the oracle, past and below one window."""
    rng = np.random.default_rng(99)
    base = stream("alternating")
    for trial in range(6):
        x = base.copy()
        for _ in range(3):
            i = 4 * int(rng.integers(0, x.size // 4))
            x[i:i + 4] = np.frombuffer(int(rng.choice([0x80000008, 0x80005000, 0x80100000, 0x00000008,
                                                       int(rng.integers(0, 1 << 32))])).to_bytes(4, "big"),
                                       dtype=np.uint8)
        for maxlen in (MS.MIB, 16380):
            want = O.index_msgs(x, maxlen)
            got = device_index(x, dev, maxlen)
            assert got[:2] == want[:2], (trial, maxlen)
            assert np.array_equal(got[2], want[2])
