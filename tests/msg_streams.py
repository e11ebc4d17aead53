"""Seeded streams of record-marked messages of any length (test helper).

A message is the 4-byte mark BE(size | 0x80000000) then `size` random
body bytes (message_t::alloc, xdrpp/marshal.cc:15-31); bodies hold random
words, some of which read as marks.  The streams are regenerated from
their seeds wherever a test runs; tests/golden/frames.json holds their
sha256 and the framing the REAL read_message / msg_sock give them
(oracle/ref_golden frame, script tests/golden/make_frames.py).
"""
from __future__ import annotations

import hashlib

import numpy as np

KIB, MIB = 1 << 10, 1 << 20
PALETTE = [0, 8, 8, 8, 100, 16380, 16384, 20 * KIB, 50000, MIB]

# name: (seed, sizes or (palette, count), edits); the edits:
#   trunc: bytes cut from the end;  frag: message whose mark loses the
#   last-fragment bit (msgsock.cc:85-91, srpc.cc:41-45)
CASES = {
    "mixed": (11, (PALETTE, 40), {}),
    "trunc_long": (12, [8, 20 * KIB, 8, MIB, 8, 16384, MIB, 8], {"trunc": 300000}),
    "frag": (13, (PALETTE, 30), {"frag": 20}),
    "alternating": (14, [8, 20 * KIB] * 300 + [8], {}),
    "long_run": (15, [16388] * 4200 + [8, 8, 8], {}),
}
# (case, max_msg_len) pairs the fixtures frame
FRAMINGS = [("mixed", MIB), ("mixed", 20 * KIB), ("mixed", 0x7FFFFFFF), ("mixed", 16380),
            ("trunc_long", MIB), ("frag", MIB), ("alternating", MIB), ("alternating", 16384),
            ("long_run", MIB)]


def sizes_of(name: str) -> list[int]:
    seed, sz, _ = CASES[name]
    if isinstance(sz, tuple):
        pal, n = sz
        rng = np.random.default_rng(seed)
        return [int(pal[i]) for i in rng.integers(0, len(pal), n)]
    return list(sz)


def stream(name: str) -> np.ndarray:
    seed, _, edits = CASES[name]
    sizes = sizes_of(name)
    rng = np.random.default_rng(seed + 1000)
    body = rng.integers(0, 256, sum(sizes) + 4 * len(sizes), dtype=np.uint8)
    pos = 0
    for k, s in enumerate(sizes):
        mark = s | (0 if edits.get("frag") == k else 0x80000000)
        body[pos:pos + 4] = np.frombuffer(mark.to_bytes(4, "big"), dtype=np.uint8)
        pos += 4 + s
    if "trunc" in edits:
        body = body[:body.size - edits["trunc"]]
    return body


def sha256(x: np.ndarray) -> str:
    return hashlib.sha256(x.tobytes()).hexdigest()
