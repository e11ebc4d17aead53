"""Regenerate tests/golden/frames.json: the framing the REAL read_message
gives the streams of tests/msg_streams.py (oracle/_ref/ref_golden frame,
built from /root/reference by `make -C oracle`).  Test infrastructure.

    python tests/golden/make_frames.py
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import msg_streams as MS  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "ref_golden")


def main() -> None:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/ref_golden"], check=True)
    out = {"generator": "oracle/ref_golden frame (read_message, srpc.cc:29-55, with msg_sock's "
                        "maxmsglen rule, msgsock.cc:97-111) over tests/msg_streams.py",
           "streams": {}, "framings": []}
    with tempfile.TemporaryDirectory() as td:
        for name in MS.CASES:
            x = MS.stream(name)
            out["streams"][name] = {"bytes": int(x.size), "sha256": MS.sha256(x)}
            path = os.path.join(td, name)
            x.tofile(path)
            for case, maxlen in MS.FRAMINGS:
                if case != name:
                    continue
                res = os.path.join(td, "r.json")
                subprocess.run([REF, "frame", path, str(maxlen), res], check=True)
                with open(res) as f:
                    r = json.load(f)
                out["framings"].append({"stream": name, "max_msg_len": maxlen, **r})
    with open(os.path.join(HERE, "frames.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
        f.write("\n")


if __name__ == "__main__":
    main()
