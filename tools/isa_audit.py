"""Audit of the pipelined encode windows in compiled code (var_kernels.h
XDRG_ENC_PIPE): the windows' payload batches are inline asm loads that the
compiler does not count, and each is waited for by an explicit, tagged
s_waitcnt vmcnt(N) after later stores (or behind the other batch).  That is
right only if, on every path of the compiled kernel, at least N vector
memory operations follow the batch's last load before its wait, and
nothing touches the batch's registers while it may be in flight.  This
compiles a plan's generated source with hipcc -save-temps and checks the
whole kernel by a dataflow over its control flow (audit()).

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


LABEL = re.compile(r"^([.\w$]+):")
TAGGED_LOAD = re.compile(r"^global_load_dwordx4\s+(v\[\d+:\d+\]),\s*(.*?)\s*;\s*xb(\d+)")
TAGGED_WAIT = re.compile(r"^s_waitcnt\s+vmcnt\((\d+)\)\s*;\s*xb(\d+)(?:\s+xb(\d+))?")
VMCNT = re.compile(r"vmcnt\((\d+)\)")
CAP = 64  # vmcnt's range: a batch with this many younger operations has landed


def parse(lines):
    """Instructions (text, is_inline_asm) and label -> index."""
    ins, labels, in_asm = [], {}, False
    for raw in lines:
        t = raw.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = LABEL.match(t)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        ins.append((t, in_asm))
    return ins, labels


def succs(ins, labels, k):
    t = ins[k][0]
    op = t.split()[0]
    if op == "s_endpgm" or op.startswith("s_setpc") or op == "s_trap":
        return []
    if op == "s_branch":
        return [labels[t.split()[1]]]
    if op.startswith("s_cbranch"):
        return [k + 1, labels[t.split()[1]]]
    return [k + 1]


def audit(lines):
    """Path-insensitive check of the asm payload batches of the encode
    windows (var_kernels.h XDRG_ENC_PIPE; loads and waits tagged "; xb<K>").
    A forward dataflow over the kernel's control flow tracks, per batch K
    that may be in flight, its destination registers and the fewest vector
    memory operations issued after its last load on any path.  Raises
    AssertionError when
      * an instruction other than the batch's own loads reads or writes a
        register of a batch that may be in flight (the value is not there
        yet, or the load would overwrite another value);
      * a tagged wait s_waitcnt vmcnt(N) ; xbK is reached with fewer than N
        younger operations behind batch K on some path (the batch would not
        have landed), or with batch K in flight on no path;
      * a batch may still be in flight at s_endpgm (a batch never read).
    A compiler s_waitcnt vmcnt(n) retires every batch with n or more
    younger operations.  Returns (waits checked, waits with N > 0: the
    loads overlap the operations after them)."""
    ins, labels = parse(lines)
    if not any(a and TAGGED_LOAD.match(t) for t, a in ins):
        return 0, 0  # no payload slots (vecrec: elements only) or XDRG_ENC_PIPE off
    n = len(ins)
    state = [None] * (n + 1)  # entry state: {tag: (regs, younger)}
    state[0] = {}
    work = [0]
    waits, effective = set(), set()

    def merge(k, st):
        old = state[k]
        if old is None:
            state[k] = st
            return True
        new = dict(old)
        for tag, (r, y) in st.items():
            if tag in new:
                r0, y0 = new[tag]
                new[tag] = (r0 | r, min(y0, y))
            else:
                new[tag] = (r, y)
        if new != old:
            state[k] = new
            return True
        return False

    def transfer(k, check):
        st = dict(state[k])
        t, is_asm = ins[k]
        pend = set().union(*(r for r, _ in st.values())) if st else set()
        ml, mw = TAGGED_LOAD.match(t), TAGGED_WAIT.match(t)
        if is_asm and ml:
            tag = int(ml.group(3))
            dst = regs(ml.group(1))
            others = set().union(*(r for g, (r, _) in st.items() if g != tag)) if st else set()
            if check:
                assert not (regs(ml.group(2)) & pend), f"load address in a batch register in flight: {t}"
                assert not (dst & others), f"batch xb{tag} loads over another batch in flight: {t}"
            st = {g: (r, min(y + 1, CAP)) for g, (r, y) in st.items() if g != tag}
            prev = state[k][tag][0] if tag in state[k] and state[k][tag][1] == 0 else frozenset()
            st[tag] = (frozenset(prev | dst), 0)
        elif is_asm and mw:
            nwait = int(mw.group(1))
            tags = [int(g) for g in mw.groups()[1:] if g]
            if check:
                assert any(g in st for g in tags), f"tagged wait with its batches in flight on no path: {t}"
                for g in tags:
                    assert g not in st or st[g][1] >= nwait, f"xb{g}: {st[g][1]} younger operations before vmcnt({nwait})"
                waits.add(k)
                if nwait:
                    effective.add(k)
            st = {g: v for g, v in st.items() if v[1] < nwait}
        else:
            if check:
                assert not (regs(t) & pend) or t.startswith("s_waitcnt"), f"batch register in flight touched: {t} (#{k}, in flight {sorted(regs(t) & pend)} of {sorted(st)})"
            m = VMCNT.search(t) if t.startswith("s_waitcnt") else None
            if m:
                st = {g: v for g, v in st.items() if v[1] < int(m.group(1))}
            elif VMEM.match(t):
                st = {g: (r, min(y + 1, CAP)) for g, (r, y) in st.items()}
        nxt = succs(ins, labels, k)
        if check and not nxt:
            assert not st, f"batch(es) {sorted(st)} in flight at {t}"
        return st, nxt

    while work:  # the fixed point first, then the checks on it
        k = work.pop()
        st, nxt = transfer(k, False)
        for j in nxt:
            if j < n and merge(j, st):
                work.append(j)
    for k in range(n):
        if state[k] is not None:
            transfer(k, True)
    assert waits, "asm loads without a tagged wait"
    return len(waits), len(effective)


def main():
    for schema in sys.argv[1:] or ["recvar", "rpc", "vecrec"]:
        with tempfile.TemporaryDirectory() as d:
            for k, lines in kernel_asm(schema, d).items():
                c, e = audit(lines)
                print(f"{schema} {k}: {c} pipelined window sequence(s) safe, {e} with the loads overlapping the stores")


if __name__ == "__main__":
    main()
