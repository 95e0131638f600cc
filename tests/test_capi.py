"""CPU: the C-ABI library loads and exports every function include/speq_scan.h declares (no compute calls)."""
import os
import re
import subprocess

from speq_amd import lib
from speq_amd._lib import ABI_VERSION, LIB_PATH, SIGNATURES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "speq_scan.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(speq_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_api():
    names = declared()
    for must in ("speq_index_build", "speq_device_open", "speq_scan_reads_device", "speq_ref_unique",
                 "speq_allreduce_u64", "speq_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (speq_[a-z0-9_]+)$", out, flags=re.M))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing


def test_python_binding_covers_header():
    assert sorted(SIGNATURES) == declared()
    L = lib()
    for name in declared():
        assert hasattr(L, name)
    assert L.speq_abi_version() == ABI_VERSION


def test_device_count_never_fails():
    assert lib().speq_device_count() >= 0
