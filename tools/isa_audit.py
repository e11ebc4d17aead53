"""Audit of the pipelined encode windows in compiled code (var_kernels.h
XDRG_ENC_PIPE): the next window's payload loads are inline asm that the
compiler does not count, and their wait is an explicit s_waitcnt vmcnt(SW)
after the window's SW buffer stores.  That wait is right only if, in the
compiled kernel, exactly the SW stores (and no other vector memory
instruction) sit between the last asm load and the wait, no compiler wait
on vmcnt sits among them, and nothing touches the loads' destination
registers before the wait.  This compiles a plan's generated source with
hipcc -save-temps and checks every such sequence.

    python tools/isa_audit.py recvar rpc vecrec
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")


def regs(text):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", text):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", text):
        out.add(int(m.group(1)))
    return out


def kernel_asm(schema, workdir):
    import ctypes as C
    from xdrpp_amd import _abi as A, build as B, schemas as S
    from xdrpp_amd.build import _Plan
    p = _Plan({**S.ALL, **S.CONTAINERS}[schema])
    L = A.lib()
    n = C.c_size_t(0)
    A.check(L.xdrg_plan_kernel_source(p.handle, None, 0, C.byref(n)), "xdrg_plan_kernel_source")
    buf = C.create_string_buffer(n.value + 1)
    A.check(L.xdrg_plan_kernel_source(p.handle, buf, n.value + 1, C.byref(n)), "xdrg_plan_kernel_source")
    src = os.path.join(workdir, f"{schema}.hip")
    with open(src, "w") as f:
        f.write(buf.value.decode())
    subprocess.check_call([B.hipcc(), "--genco", f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-save-temps",
                           "-I", B.CSRC, "-I", os.path.join(ROOT, "include"), "-o", os.path.join(workdir, "x.co"),
                           src], cwd=workdir)
    s = open([os.path.join(workdir, f) for f in os.listdir(workdir)
              if f.startswith(schema) and f.endswith(".s") and "gfx" in f][0]).read()
    out = {}
    for k in ("xdrg_spec_encode", "xdrg_spec_encode_pre", "xdrg_spec_encode_lb"):
        if f"\n{k}:" in s:
            i = s.index(f"\n{k}:")
            out[k] = s[i:s.index(".Lfunc_end", i)].splitlines()
    return out


def audit(lines):
    """(sequences checked, sequences whose loads really overlap the stores).
    Raises AssertionError when a wait could let a load's data be read early:
    fewer stores between the last asm load and its vmcnt(N) than N, or a
    destination register touched before the wait.  A compiler vmcnt(0)
    among them is safe (it waits for the asm loads too) but defeats the
    overlap; it is counted as not effective."""
    ins = [ln.strip() for ln in lines]
    # the batch's asm loads: 16-byte chunks and (XDRG_ENC_ALIGN) the word after each
    asm_loads = [k for k, t in enumerate(ins) if t.startswith("global_load_dword") and k > 0
                 and ins[k - 1] == ";;#ASMSTART"]
    if not asm_loads:
        return 0, 0  # no payload slots (vecrec: elements only) or XDRG_ENC_PIPE off
    checked = effective = 0
    for k in asm_loads:
        nxt = [j for j in asm_loads if j > k]
        if nxt and not any(VMEM.match(ins[j]) or ins[j].startswith("s_waitcnt vmcnt") for j in range(k + 1, nxt[0])):
            continue  # not the batch's last load
        group = [j for j in asm_loads if j <= k and j >= k - 80]
        dsts = set().union(*(regs(ins[j].split(",")[0]) for j in group))
        stores, wait, covered = 0, None, False
        for j in range(k + 1, len(ins)):
            t = ins[j]
            if not t or t.startswith(";") or t.startswith("."):
                continue
            m = re.match(r"s_waitcnt vmcnt\((\d+)\)", t)
            if m and ins[j - 1] == ";;#ASMSTART":
                wait = int(m.group(1))
                break
            if m:
                assert int(m.group(1)) == 0 or covered, f"compiler partial vmcnt wait among the stores: {t}"
                covered = True
                continue
            if VMEM.match(t):
                assert t.startswith("buffer_store_dwordx4"), f"other memory op before the wait: {t}"
                stores += 1
            elif regs(t) & dsts and not covered and not t.startswith("buffer_store"):
                raise AssertionError(f"asm load destination touched before its wait: {t}")
            # branches allowed: the skip of the wait when nothing was
            # prefetched, after every store (the fall-through reaches the
            # wait), and a forward skip over straight-line code that is
            # itself scanned here (an LDS read of one lane: its target is a
            # label before the wait)
            if t.startswith("s_cbranch") and stores == 0:
                target = t.split()[-1]
                rest = ins[j + 1:]
                lab = next((q for q, x in enumerate(rest) if x.startswith(target + ":")), None)
                waits = [q for q, x in enumerate(rest) if re.match(r"s_waitcnt vmcnt\(\d+\)", x)
                         and rest[q - 1] == ";;#ASMSTART"]
                assert lab is not None and waits and lab < waits[0], f"branch among the loads and stores: {t}"
        assert wait is not None and (covered or stores == wait), f"{stores} stores before vmcnt({wait})"
        checked += 1
        effective += not covered
    assert checked, "asm loads without a load/store/wait sequence"
    return checked, effective


def main():
    for schema in sys.argv[1:] or ["recvar", "rpc", "vecrec"]:
        with tempfile.TemporaryDirectory() as d:
            for k, lines in kernel_asm(schema, d).items():
                c, e = audit(lines)
                print(f"{schema} {k}: {c} pipelined window sequence(s) safe, {e} with the loads overlapping the stores")


if __name__ == "__main__":
    main()
