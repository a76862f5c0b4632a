"""CPU: the product's device headers (at2-node_amd/csrc/*.h) compiled for the HOST with g++ and run
over every golden fixture, both policies. This checks the field/group/scalar/SHA code paths before
any GPU is involved. It is a test build only: the shipped path is the HIP kernel in libat2v.so."""
import os
import subprocess

import pytest

import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "host", "verify_host.cpp")
EXE = os.path.join(ROOT, "tests", "host", "verify_host")


INC = "-I" + os.path.join(ROOT, "at2-node_amd", "csrc")
BUILDS = {  # the plain build and the sanitized one (-O0: the always-inline field code takes minutes at -O1 under ASan)
    EXE: ["g++", "-O2", "-std=c++17", INC, SRC],
    EXE + "_asan": ["g++", "-O0", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", INC, SRC],
}


@pytest.fixture(scope="module")
def host_exes():
    """both builds, compiled CONCURRENTLY (each takes ~2.5 min), each to a per-process name and then renamed into place,
    so parallel test workers (pytest -n) never execute a file another worker is still writing"""
    procs = {exe: subprocess.Popen(cmd + ["-o", f"{exe}.{os.getpid()}"]) for exe, cmd in BUILDS.items()}
    for exe, pr in procs.items():
        assert pr.wait() == 0, f"build of {exe} failed"
        os.replace(f"{exe}.{os.getpid()}", exe)
    return list(BUILDS)


@pytest.fixture(scope="module")
def host_exe(host_exes):
    return host_exes[0]


@pytest.fixture(scope="module")
def host_exe_asan(host_exes):
    return host_exes[1]


MODES = [0, 1, 2, 3, 4, 5, 6]
MODE_IDS = ["full_length", "half_size", "half_size_unsigned_field", "two_lanes_per_record", "sender_comb",
            "sender_comb_split", "four_wave_split_half_size"]


@pytest.mark.parametrize("half", MODES, ids=MODE_IDS)
def test_sanitized_host_build_of_device_core(host_exe_asan, half):
    """the same code under AddressSanitizer + UBSan (signed overflow, shifts, bounds) over the edge and
    adversarial fixtures (the comb form on fewer records: every distinct key builds its 4128-entry comb)"""
    for name, limit in (("edge", 3000), ("adversarial", 800)):
        if half >= 4:
            limit = 40
        out = subprocess.run([host_exe_asan, os.path.join(golden_io.GOLDEN_DIR, name + ".bin"), str(limit), str(half)],
                             capture_output=True, text=True, timeout=900)
        assert out.returncode == 0, out.stderr[-3000:]


@pytest.mark.parametrize("half", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("name", golden_io.SETS)
def test_host_build_of_device_core_matches_golden(host_exe, name, half):
    """every verify form the kernels can be built with: the full-length ladder (verify_core), the half-size lattice
    form on the signed field (verify_half) and on the unsigned chained-carry field (verify_half_fu, the throughput
    kernel), its two-lanes-per-record split (verify_pair_part + verify_pair_combine, the low-latency kernel), and the
    sender-comb form (comb_build_lane + verify_comb_fu, at2v_comb.h) and its low-latency four-wave split (comb_decode_r,
    comb_sum over the halves, comb_check_split) on the first 1,200 records of a set (every distinct key builds its
    comb), against OpenSSL/libsodium-derived verdicts"""
    limit = "1200" if half >= 4 else "1000000"
    out = subprocess.run([host_exe, os.path.join(golden_io.GOLDEN_DIR, name + ".bin"), limit, str(half)],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    n, bad_d, bad_s = map(int, out.stdout.split())
    assert bad_d == 0 and bad_s == 0 and n > 0


def test_unsigned_field_bounds_at_class_extremes():
    """the unsigned-field group law (at2v_gu.h) on maximal-limb inputs with every operand and column checked
    (-DAT2V_FU_CHECK), plus value checks of the formulas from such representatives"""
    exe = os.path.join(ROOT, "tests", "host", "fu_bounds_host")
    subprocess.run(["g++", "-O1", "-std=c++17", "-DAT2V_FU_CHECK", "-I" + os.path.join(ROOT, "at2-node_amd", "csrc"),
                    os.path.join(ROOT, "tests", "host", "fu_bounds_host.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stderr[-2000:]


def test_unsigned_field_generator_is_current():
    """at2v_fu_gen.h must be what tools/gen_fu.py (bound proof + group-law model) emits."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "g.h")
        subprocess.run(["python3", os.path.join(ROOT, "tools", "gen_fu.py"), p], check=True, capture_output=True)
        assert open(p).read() == open(os.path.join(ROOT, "at2-node_amd", "csrc", "at2v_fu_gen.h")).read()


def test_field_bounds_generator_is_current():
    """at2v_fe_gen.h must be what tools/gen_fe.py (the bound proof) emits."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "g.h")
        subprocess.run(["python3", os.path.join(ROOT, "tools", "gen_fe.py"), p], check=True, capture_output=True)
        assert open(p).read() == open(os.path.join(ROOT, "at2-node_amd", "csrc", "at2v_fe_gen.h")).read()
