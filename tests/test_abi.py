"""CPU checks of the C-ABI library: it loads without a GPU, exports every symbol the
headers in include/ declare, its host-side matrix code (reed_sol / jerasure_invert)
agrees with the oracle, and every compute entry point fails loudly (no CPU fallback)
when there is no GPU."""
from __future__ import annotations

import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ["cocytus_ec.h", "galois.h", "jerasure.h", "reed_sol.h"]


def declared_functions() -> set[str]:
    names = set()
    for h in HEADERS:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b([a-z_][a-z0-9_]*)\s*\(", src):
            name = m.group(1)
            if name.startswith(("cec_", "galois_", "reed_sol_", "jerasure_")):
                names.add(name)
    return names


@pytest.fixture(scope="module")
def lib():
    from cocytus_amd import build, ec

    build.build(verbose=False)
    return ec


def exported_symbols(path: str) -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True)
    return {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}


def test_exports_every_declared_symbol(lib):
    decl = declared_functions()
    assert {"galois_w08_region_multiply", "reed_sol_big_vandermonde_distribution_matrix",
            "jerasure_invert_matrix", "cec_encode", "cec_decode", "cec_diff_update"} <= decl
    syms = exported_symbols(lib.LIB_PATH)
    missing = decl - syms
    assert not missing, missing
    lib.lib()  # every binding resolves
    # -lJerasure drop-in name
    assert os.path.realpath(os.path.join(ROOT, "cocytus_amd", "libJerasure.so")) == os.path.realpath(lib.LIB_PATH)


def test_no_internal_symbols_leak(lib):
    syms = exported_symbols(lib.LIB_PATH)
    ours = {s for s in syms if not s.startswith(("cec_", "galois_", "reed_sol_", "jerasure_", "_"))}
    assert not {s for s in ours if "combine" in s or "cec" in s.lower()}


@pytest.mark.parametrize("k,m", [(1, 1), (2, 1), (3, 2), (4, 2), (6, 3), (10, 4), (12, 8), (16, 16)])
def test_coding_matrix_matches_oracle(lib, oracle, k, m):
    assert lib.reed_sol_big_vandermonde_distribution_matrix(k + m, k, 8) == oracle.big_vandermonde(k + m, k)


def test_coding_matrix_known_answers(lib):
    # SURVEY.md §8c restated known answers (parity rows only)
    assert lib.coding_matrix(3, 2)[9:] == [1, 1, 1, 1, 245, 244]
    assert lib.coding_matrix(4, 2)[16:] == [1, 1, 1, 1, 1, 70, 143, 200]
    assert lib.reed_sol_big_vandermonde_distribution_matrix(3, 3, 8) is None
    assert lib.reed_sol_big_vandermonde_distribution_matrix(5, 3, 16) is None


def test_invert_matches_oracle(lib, oracle):
    import numpy as np

    rng = np.random.default_rng(9)
    for n in [1, 2, 3, 4, 6, 8]:
        for _ in range(30):
            mat = [int(x) for x in rng.integers(0, 256, n * n)]
            if rng.random() < 0.2:
                mat[: n] = [0] * n  # singular
            r1, inv1 = lib.jerasure_invert_matrix(mat, n, 8)
            r2, inv2 = oracle.invert(mat, n)
            assert r1 == r2
            if r1 == 0:
                assert inv1 == inv2


def test_single_ops(lib, oracle):
    for a in range(0, 256, 7):
        for b in range(0, 256, 5):
            assert lib.galois_single_multiply(a, b, 8) == oracle.gf_mul(a, b)
            assert lib.galois_single_divide(a, b, 8) == oracle.gf_div(a, b)


def test_compute_fails_loudly_without_gpu(lib):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    assert lib.device_check() == lib.CEC_ENODEV
    with pytest.raises(lib.CecError) as ei:
        lib.Plan([(0, 0, 4096, 0)])
    assert ei.value.code == lib.CEC_ENODEV
    with pytest.raises(lib.CecError):
        lib.region_multiply(0x1000, 2, 16, 0x2000, 1)
    with pytest.raises(lib.CecError):
        lib.encode_region(3, 2, lib.coding_matrix(3, 2), [0x1000] * 3, [0x2000] * 2, 4096)
    # the void drop-in aborts with a message instead of computing on the CPU
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np\nfrom cocytus_amd import ec\n"
            "a = np.ones(64, np.uint8); b = np.zeros(64, np.uint8)\n"
            "ec.galois_w08_region_multiply(a, 2, 64, b, 1)\nprint('computed')\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "computed" not in r.stdout
    assert "libcocytus_ec: fatal" in r.stderr


def test_bad_arguments_rejected(lib):
    mat = lib.coding_matrix(3, 2)
    with pytest.raises(lib.CecError) as ei:
        lib.encode_region(0, 2, mat, [], [0, 0], 16)
    assert ei.value.code == lib.CEC_EINVAL
    with pytest.raises(lib.CecError) as ei:
        lib.encode_region(17, 2, [1] * 19 * 17, [0] * 17, [0, 0], 16)
    assert ei.value.code == lib.CEC_EINVAL
    assert lib.recovery_mask(3, 2, 3, [1, 1, 1, 1, 1]) == 0b01011
    assert lib.recovery_mask(3, 2, 3, [0, 0, 1, 1, 0]) == 0


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (6, 3)])
def test_recovery_mask_matches_oracle_every_pattern(lib, oracle, k, m):
    """cec_recovery_mask == start_recovery's selection (memcached.c:8136-8151, via the
    oracle) for every leader and every connectivity pattern; host logic, no GPU."""
    import itertools

    for leader in range(k + m):
        for conn in itertools.product([0, 1], repeat=k + m):
            conn = list(conn)
            assert lib.recovery_mask(k, m, leader, conn) == oracle.recovery_mask(k, m, leader, conn)


def test_arena_stride_is_odd_pages(lib):
    """cec_arena_stride: an odd number of 4 KiB pages covering the arena."""
    for n in [1, 4095, 4096, 8192, 12288, (256 << 20), (256 << 20) + 1, 3 * 4096 + 5]:
        s = lib.arena_stride(n)
        assert s >= n and s % 4096 == 0 and (s // 4096) % 2 == 1 and s - n < 2 * 4096


def test_default_engine_is_auto(lib):
    """The product default is AUTO: the LDS engine only where it led PERM by more than 2 %
    on the median of the recorded boxes -- cec_decode of values of 64 KiB and more -- and
    PERM for every other op (cocytus_ec.h, DESIGN.md §4;
    the choices themselves are asserted on the GPU, test_auto_engine_choices).  PERM and
    LDS stay selectable and both are in every GPU parity test; AUTO is what every test
    that leaves the engine alone runs."""
    assert lib.get_engine() == lib.CEC_ENGINE_AUTO
    assert lib.last_engine() == -1  # no op has run on this thread
    for e in (lib.CEC_ENGINE_PERM, lib.CEC_ENGINE_LDS, lib.CEC_ENGINE_AUTO):
        lib.set_engine(e)
        assert lib.get_engine() == e
    with pytest.raises(lib.CecError):
        lib.set_engine(3)


def test_waves_per_cu_knob(lib):
    """Occupancy cap: off by default (DESIGN.md §4 measured it and kept it off), settable,
    range-checked; no device is needed to set it."""
    import os

    if not os.environ.get("CEC_WAVES_PER_CU"):
        assert lib.get_waves_per_cu() == 0
    before = lib.get_waves_per_cu()
    lib.set_waves_per_cu(16)
    assert lib.get_waves_per_cu() == 16
    with pytest.raises(lib.CecError):
        lib.set_waves_per_cu(-1)
    lib.set_waves_per_cu(before)


def test_headers_are_c99_and_cxx(tmp_path):
    """include/*.h compile as strict C99 (the reference server is C) and as C++."""
    src = tmp_path / "h.c"
    src.write_text("".join(f"#include <{h}>\n" for h in HEADERS) + "int main(void) { return 0; }\n")
    inc = os.path.join(ROOT, "include")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", inc, "-c", str(src),
                    "-o", str(tmp_path / "h.o")], check=True)
    subprocess.run(["g++", "-std=c++11", "-Wall", "-Werror", "-I", inc, "-x", "c++", "-c", str(src),
                    "-o", str(tmp_path / "hpp.o")], check=True)


LLVM_OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


@pytest.mark.skipif(not os.path.exists(LLVM_OBJDUMP), reason="llvm-objdump not in this image")
def test_release_epilogue_in_gfx950_code(lib, tmp_path):
    """Round 2's stale-tile defect, checked in the shipped machine code on any host: every
    kSysRel instantiation of combine_kernel (the drop-in's host-visible launches) ends each
    wave with the system-scope L2 writeback `buffer_wbl2 sc0 sc1` followed by
    `s_waitcnt vmcnt(0)` before `s_endpgm`, with nothing in between; no other combine
    kernel writes back L2 (the batched kernels pay nothing).  The GPU tests assert the
    host side (which launches get it, cec_last_sync)."""
    import shutil

    so = tmp_path / "lib.so"
    shutil.copy(os.path.realpath(lib.LIB_PATH), so)
    subprocess.run([LLVM_OBJDUMP, "--offloading", str(so)], cwd=tmp_path, check=True,
                   capture_output=True)
    cos = [p for p in tmp_path.iterdir() if p.name.endswith("gfx950")]
    assert len(cos) == 1, sorted(p.name for p in tmp_path.iterdir())
    dis = subprocess.run([LLVM_OBJDUMP, "-d", str(cos[0])], check=True, capture_output=True,
                         text=True).stdout
    funcs: dict[str, list[str]] = {}
    cur = None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur and line.startswith("\t") and not line.startswith("\t\t"):
            funcs[cur].append(line.split("//")[0].strip())
    combine = {f: ins for f, ins in funcs.items() if "combine_kernel" in f}
    assert len(combine) > 50, len(combine)
    released = {}
    for f, ins in combine.items():
        m = re.search(r"Lb([01])EEEvNS_12CombineArgsN", f)
        assert m, f
        released[f] = m.group(1) == "1"
    sysrel = [f for f, r in released.items() if r]
    # the narrow 1 x 1 kernels: both engines x (write, XOR-accumulate)
    assert len(sysrel) == 4 and {("Perm" in f, "ELi1ELb1ELi2" in f) for f in sysrel} == {
        (p, a) for p in (True, False) for a in (True, False)}, sysrel
    for f, ins in combine.items():
        wb = [i for i in ins if i.startswith("buffer_wbl2")]
        ends = [k for k, i in enumerate(ins) if i == "s_endpgm"]
        assert ends, f
        if not released[f]:
            assert not wb, (f, wb)
            continue
        for e in ends:
            k = e - 1
            while ins[k] == "s_waitcnt vmcnt(0)":
                k -= 1
            assert k < e - 1 and ins[k] == "buffer_wbl2 sc0 sc1", (f, ins[max(0, e - 6):e + 1])


def test_launch_layout_check_refuses(lib):
    """The launch-time check (cocytus_ec.h test hook, the very function every launch runs):
    a pattern naming a stream slot the kernel's argument block does not carry -- slot 2 on
    the two-slot narrow 1 x 1 kernels -- or a slot whose base is NULL is refused with
    CEC_EINVAL before anything is launched (no device needed); a block that serves the
    pattern passes."""
    a, b, c = 0x10000, 0x20000, 0x30000
    ok, bad = lib.CEC_OK, lib.CEC_EINVAL
    # narrow: two slots only
    assert lib.check_launch_layout(True, [0], [1], [a, b]) == ok
    assert lib.check_launch_layout(True, [0], [2], [a, b, c]) == bad  # slot 2 is not in the block
    assert lib.check_launch_layout(True, [2], [1], [a, b, c]) == bad
    assert lib.check_launch_layout(True, [0], [1], [a, None]) == bad  # NULL output base
    # the full block: every slot the pattern names must hold a base
    assert lib.check_launch_layout(False, [0, 1, 2], [3, 4], [a, b, c, a + 1, b + 1]) == ok
    assert lib.check_launch_layout(False, [0, 1, 2], [3, 5], [a, b, c, a + 1, b + 1]) == bad
    assert lib.check_launch_layout(False, [0, 9], [3], [a, b, c, a + 1]) == bad
    assert "not launched" in lib.lib().cec_last_error().decode()


def _policy_in_child(env_extra):
    env = dict(os.environ)
    for k in ("CEC_STORE_POLICY", "CEC_WT_MAX_BYTES"):
        env.pop(k, None)
    env.update(env_extra)
    code = ("import sys, json; sys.path.insert(0, %r)\nfrom cocytus_amd import ec\n"
            "print(json.dumps(ec.store_policy()))\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    import json

    return tuple(json.loads(r.stdout.strip().splitlines()[-1])), r.stderr


def test_store_policy_environment(lib):
    """CEC_STORE_POLICY / CEC_WT_MAX_BYTES (measurement overrides of the per-launch store
    policy): nt, wt and auto are taken; anything else (e.g. "WT") is reported
    on stderr and means auto, instead of silently selecting non-temporal stores."""
    assert _policy_in_child({}) == (("auto", 512 << 20), "")
    assert _policy_in_child({"CEC_STORE_POLICY": "nt"})[0] == ("nt", 512 << 20)
    assert _policy_in_child({"CEC_STORE_POLICY": "wt"})[0] == ("wt", 512 << 20)
    assert _policy_in_child({"CEC_WT_MAX_BYTES": "0"})[0] == ("auto", 0)
    got, err = _policy_in_child({"CEC_STORE_POLICY": "WT"})
    assert got == ("auto", 512 << 20) and "CEC_STORE_POLICY=WT" in err
    got, err = _policy_in_child({"CEC_WT_MAX_BYTES": "lots"})
    assert got == ("auto", 512 << 20) and "CEC_WT_MAX_BYTES=lots" in err
    # strtoull would read "-1" as 2^64 - 1 (write-through for every launch) and skip blanks;
    # neither is a byte count, nor is a value past 2^64 - 1
    for bad in ("-1", " 4096", "+4096", "99999999999999999999999"):
        got, err = _policy_in_child({"CEC_WT_MAX_BYTES": bad})
        assert got == ("auto", 512 << 20) and "CEC_WT_MAX_BYTES=" in err, bad
    assert _policy_in_child({"CEC_WT_MAX_BYTES": "0x1000"})[0] == ("auto", 4096)


@pytest.mark.skipif(not os.path.exists(LLVM_OBJDUMP), reason="llvm-objdump not in this image")
def test_kernel_code_id(lib):
    """ec.kernel_code_id: a stable identity of the library's gfx950 kernels (their
    disassembly, by name), the key bench.py uses to decide whether the committed PMC
    traffic still describes the kernels it runs."""
    a = lib.kernel_code_id()
    assert a and re.fullmatch(r"[0-9a-f]{16}", a)
    assert lib.kernel_code_id() == a
    assert lib.kernel_code_id("/nonexistent/lib.so") is None


def test_roofline_traffic_tied_to_the_build(tmp_path, monkeypatch):
    """bench.py reports roofline.traffic from profiles/pmc_traffic*.json only while the
    summary's recorded kernel_code_id equals the library's; otherwise (or with no record)
    traffic is null and traffic_stale is true."""
    import json

    import bench

    prof = tmp_path / "profiles"
    prof.mkdir()
    doc = {"rs32_4k": {"encode_hbm_bytes_per_launch": 11.0, "decode_hbm_bytes_per_launch": 22.0},
           "_build": {"kernel_code_id": "00112233aabbccdd"}}
    (prof / "pmc_traffic.json").write_text(json.dumps(doc))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.load_traffic("rs32_4k", code_id="00112233aabbccdd") == ((11.0, 22.0), False)
    assert bench.load_traffic("rs32_4k", code_id="ffffffffffffffff") == ((None, None), True)
    assert bench.load_traffic("rs32_4k", ("encode",), "lds", code_id="00112233aabbccdd") == ((None,), True)
    del doc["_build"]
    (prof / "pmc_traffic.json").write_text(json.dumps(doc))
    assert bench.load_traffic("rs32_4k", code_id="00112233aabbccdd") == ((None, None), True)


def test_host_batch_wave_planning(tmp_path):
    """cec_region_multiply_batch's planning (cec_hostbatch.inc: the pieces, the range-assign
    / range-max tree and hb_cluster_waves), spliced from the shipped source into
    tests/drain_c/hb_waves_main.cpp and run under ASan + UBSan on 4,000 random clusters:
    overlapping pieces never share a wave, a cluster holding a write keeps job order, an
    XOR-only cluster takes exactly its overlap depth in waves."""
    src = open(os.path.join(ROOT, "cocytus_amd", "csrc", "cec_hostbatch.inc")).read()
    a, b = src.index("enum HbKind"), src.index("struct HbCopy {")
    prog = open(os.path.join(ROOT, "tests", "drain_c", "hb_waves_main.cpp")).read()
    cpp = tmp_path / "hb_waves.cpp"
    cpp.write_text(prog.replace("// HB_FUNCS", src[a:b]))
    exe = tmp_path / "hb_waves"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-o", str(exe), str(cpp)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr[-2000:]


def test_drain_wave_colouring(tmp_path):
    """The drainer's host-side colouring (cec_drain.inc: the radix address sort and the
    greedy interval colouring with its no-overlap fast path), spliced from the shipped
    source into tests/drain_c/waves_main.cpp and run under ASan + UBSan on 3,000 random
    batches: overlapping updates never share a launch wave, distinct values take one."""
    src = open(os.path.join(ROOT, "cocytus_amd", "csrc", "cec_drain.inc")).read()
    a, b = src.index("static void sort_by_addr("), src.index("CEC_API int cec_drainer_apply(")
    prog = open(os.path.join(ROOT, "tests", "drain_c", "waves_main.cpp")).read()
    cpp = tmp_path / "waves.cpp"
    cpp.write_text(prog.replace("// WAVES_FUNCS", src[a:b]))
    exe = tmp_path / "waves"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-o", str(exe), str(cpp)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr[-2000:]
