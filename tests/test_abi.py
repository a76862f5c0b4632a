"""CPU: the C-ABI library loads and exports every symbol include/at2v.h declares (no compute calls)."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "at2v.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(at2v_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    import at2v
    if not os.path.exists(at2v.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "at2-node_amd")], check=True)
    return at2v.load_library()


def test_header_declares_expected_api():
    import at2v
    assert declared_functions() == sorted(at2v.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (at2v_[a-z0-9_]+)", out))
    assert exported == set(declared_functions())


def test_strerror_codes(lib):
    import at2v
    assert at2v.strerror(0) == "ok"
    assert at2v.strerror(-5) == "misaligned device pointer"
    assert at2v.strerror(-99) == "unknown error"


def test_invalid_arguments_rejected_without_device(lib):
    assert lib.at2v_create(None, None) == -1
    assert lib.at2v_verify_batch(None, None, None, None, None, 0, None) == -1
    assert lib.at2v_verify_one(None, None, None, 0) == -1


def test_library_contains_gfx950_code_object(lib):
    blob = open(lib._name, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="checks the no-GPU error path")
def test_no_device_fails_loudly():
    code = ("import sys; sys.path.insert(0, %r); import at2v\n"
            "try:\n    at2v.BatchVerifier()\nexcept at2v.At2vError as e:\n    print('ERR', e.code)\n") % os.path.join(
        ROOT, "at2-node_amd")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert "ERR -2" in out.stdout, out.stdout + out.stderr
