"""The xdrc wiring of the plan back end:
`xdrpp_amd/gen/xdrc_plan.patch` adds `-plan`, `-kernels DIR` and
`-validate E1,E2` to the reference's own xdrc (`xdrc/xdrc.cc:103-192`: the
option table, the `void (*gen)(std::ostream &)` mode switch, the output
suffix) and gen_plan.cc to its build (`Makefile.am:5-19`).

CPU, in a scratch copy of the pristine reference files:
* the patch applies (`patch --dry-run`, then for real);
* the patched xdrc.cc compiles with the reference's gen_hh.cc and
  gen_server.cc and the product's gen_plan.cc, and its main() runs: its
  front end is oracle/xdrc_front_stub.cc (flex/bison are not in the image:
  yyparse() reads the cpp output and fills the AST oracle/xdrc_front.py
  built for the same file), everything else is xdrc.cc's own code;
* `xdrc -plan` writes the plan header oracle/xdrc_driver.cc writes
  (the one tests/test_gen_plan.py pins against the Python compiler and the
  recorded xdr_traits plans), `-validate` opts enums in, `-kernels DIR`
  writes the kernel sources, `-o` names the guards as gen_hh's do, and
  `-hh` is untouched.
Needs /root/reference (in this container only) and oracle/_ref/gen
(`make -C oracle`)."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference"
GEN = os.path.join(ROOT, "oracle", "_ref", "gen")
PATCH = os.path.join(ROOT, "xdrpp_amd", "gen", "xdrc_plan.patch")
STUB = os.path.join(ROOT, "oracle", "xdrc_front_stub.cc")
LIB = os.path.join(ROOT, "xdrpp_amd")

pytestmark = pytest.mark.skipif(
    not (os.path.exists(os.path.join(REF, "xdrc", "xdrc.cc")) and
         os.path.exists(os.path.join(GEN, "gen_hh.o")) and shutil.which("patch")),
    reason="needs /root/reference, oracle/_ref/gen (make -C oracle) and patch")

CXX = ["g++", "-std=c++20", "-O1", "-DXDRPP_WORDS_BIGENDIAN=0"]


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    """A scratch copy of the pristine xdrc/ and Makefile.am with the patch
    applied, and the patched xdrc built once per AST (xdrtest, validated)."""
    d = tmp_path_factory.mktemp("xdrc_patch")
    shutil.copytree(os.path.join(REF, "xdrc"), d / "xdrc")
    shutil.copy(os.path.join(REF, "Makefile.am"), d / "Makefile.am")
    dry = subprocess.run(["patch", "-p1", "--dry-run", "-i", PATCH], cwd=d, capture_output=True, text=True)
    assert dry.returncode == 0, dry.stdout + dry.stderr
    assert "FAILED" not in dry.stdout and "offset" not in dry.stdout.lower(), dry.stdout
    subprocess.check_call(["patch", "-p1", "-s", "-i", PATCH], cwd=d)
    # xdrpp/config.h is configure output (PACKAGE_VERSION, CPP_COMMAND: configure.ac)
    (d / "cfg" / "xdrpp").mkdir(parents=True)
    (d / "cfg" / "xdrpp" / "config.h").write_text('#define PACKAGE_VERSION "0-plan"\n#define CPP_COMMAND "cpp"\n')
    inc = ["-I", str(d / "cfg"), "-I", REF, "-I", os.path.join(REF, "xdrc"), "-I", os.path.join(ROOT, "xdrpp_amd", "gen"),
           "-I", os.path.join(ROOT, "include")]
    objs = []
    for src in (str(d / "xdrc" / "xdrc.cc"), os.path.join(REF, "xdrc", "gen_server.cc"), STUB,
                os.path.join(ROOT, "xdrpp_amd", "gen", "gen_plan.cc")):
        o = str(d / (os.path.basename(src) + ".o"))
        subprocess.check_call(CXX + inc + ["-c", "-o", o, src])
        objs.append(o)
    bins = {}
    for name in ("xdrtest", "validated"):
        ast = os.path.join(GEN, f"{name}_ast.cc")
        if not os.path.exists(ast):
            pytest.skip(f"{ast} not built")
        b = str(d / f"xdrc_{name}")
        subprocess.check_call(CXX + inc + ["-o", b, ast] + objs + [os.path.join(GEN, "gen_hh.o"),
                                                                   "-L", LIB, "-lxdrgpu", f"-Wl,-rpath,{LIB}"])
        bins[name] = b
    return d, bins


def run(b, args, cwd):
    return subprocess.run([b] + args, cwd=cwd, capture_output=True, text=True)


def test_patch_touches_only_the_mode_table_and_build(tree):
    d, _ = tree
    text = open(PATCH).read()
    files = re.findall(r"^\+\+\+ b/(\S+)", text, re.M)
    assert files == ["xdrc/xdrc.cc", "Makefile.am"]
    patched = (d / "xdrc" / "xdrc.cc").read_text()
    for want in ('{"plan", no_argument, nullptr, OPT_PLAN}', '{"kernels", required_argument, nullptr, OPT_KERNELS}',
                 "gen = gen_plan_mode;", 'suffix = "_plan.hh";', "xdrg_gen::gen_plan(os, symlist, plan_opts)"):
        assert want in patched
    mk = (d / "Makefile.am").read_text()
    assert "gen_plan.cc" in mk and "-lxdrgpu" in mk


def test_plan_mode_equals_driver(tree):
    """xdrc -plan over xdrtest.x = the header the oracle's driver emits (and
    tests/test_gen_plan.py pins); -hh is still gen_hh's genuine header."""
    d, bins = tree
    shutil.copy(os.path.join(REF, "tests", "xdrtest.x"), d / "xdrtest.x")
    got = run(bins["xdrtest"], ["-plan", "-o", "-", "xdrtest.x"], d)
    assert got.returncode == 0, got.stderr
    want = subprocess.run([os.path.join(GEN, "xdrcplan_xdrtest"), "-plan", "xdrtest.x"], capture_output=True,
                          text=True, check=True).stdout
    assert got.stdout == want
    hh = run(bins["xdrtest"], ["-hh", "-o", "-", "xdrtest.x"], d)
    genuine = subprocess.run([os.path.join(GEN, "xdrc_xdrtest"), "xdrtest.x"], capture_output=True, text=True,
                             check=True).stdout
    assert hh.returncode == 0 and hh.stdout == genuine


def test_validate_option(tree):
    d, bins = tree
    shutil.copy(os.path.join(ROOT, "oracle", "x", "validated.x"), d / "validated.x")
    got = run(bins["validated"], ["-plan", "-validate", "other_color", "-o", "-", "validated.x"], d)
    assert got.returncode == 0, got.stderr
    want = subprocess.run([os.path.join(GEN, "xdrcplan_validated"), "-plan", "-validate", "other_color",
                           "validated.x"], capture_output=True, text=True, check=True).stdout
    assert got.stdout == want
    plain = run(bins["validated"], ["-plan", "-o", "-", "validated.x"], d)
    assert plain.returncode == 0 and plain.stdout != want  # the opt-in changes the plan


def test_kernels_option_and_default_output(tree):
    """-kernels DIR writes each variable-length type's source (the ones the
    oracle build compiled are equal); the default output is file_plan.hh
    with the guards of xdrc's naming."""
    d, bins = tree
    shutil.copy(os.path.join(REF, "tests", "xdrtest.x"), d / "xdrtest.x")
    (d / "k").mkdir(exist_ok=True)
    got = run(bins["xdrtest"], ["-plan", "-kernels", "k", "xdrtest.x"], d)
    assert got.returncode == 0, got.stderr
    out = (d / "xdrtest_plan.hh").read_text()
    assert "#ifndef __XDR_XDRTEST_PLAN_HH_INCLUDED__" in out
    assert "__XDR_XDRTEST_HH_INCLUDED__" in out  # the -hh header's guard: emitted_plan<T> follows it
    for name in ("testns_hasbytes.hip", "testns_containertest.hip"):
        assert (d / "k" / name).read_text() == open(os.path.join(GEN, "plan", "kernels", name)).read()
    assert (d / "k" / "test_recursive.hip").exists()


def test_output_name_sets_guards(tree):
    """-o proto/x_plan.hh: the plan guard from that name, the -hh guard from
    proto/x.hh, exactly what `xdrc -hh -o proto/x.hh` puts in its header."""
    d, bins = tree
    shutil.copy(os.path.join(REF, "tests", "xdrtest.x"), d / "xdrtest.x")
    (d / "proto").mkdir(exist_ok=True)
    assert run(bins["xdrtest"], ["-plan", "-o", "proto/x_plan.hh", "xdrtest.x"], d).returncode == 0
    assert run(bins["xdrtest"], ["-hh", "-o", "proto/x.hh", "xdrtest.x"], d).returncode == 0
    plan = (d / "proto" / "x_plan.hh").read_text()
    hh = (d / "proto" / "x.hh").read_text()
    hh_guard = re.search(r"#ifndef (__XDR_\w+__)", hh).group(1)
    assert hh_guard == "__XDR_PROTO_X_HH_INCLUDED__"
    assert "#ifndef __XDR_PROTO_X_PLAN_HH_INCLUDED__" in plan
    assert hh_guard in plan


def test_mode_conflicts_and_usage(tree):
    d, bins = tree
    shutil.copy(os.path.join(REF, "tests", "xdrtest.x"), d / "xdrtest.x")
    bad = run(bins["xdrtest"], ["-plan", "-hh", "xdrtest.x"], d)
    assert bad.returncode == 1 and "usage: xdrc MODE" in bad.stderr
    h = run(bins["xdrtest"], ["-help"], d)
    assert h.returncode == 0 and "-plan" in h.stdout and "-kernels DIR" in h.stdout
