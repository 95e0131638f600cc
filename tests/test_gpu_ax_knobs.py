"""GPU: every compile-time knob of k_scan_ax forced to a non-default value still gives the oracle's counts.

The knobs (ax_scan.hip's header lists them) are A/B switches; a build that flips one must not change a result. `make
axknobs` compiles three variant libraries that together move every knob off its default (AXKNOB_VARIANTS in the
Makefile); each runs tests/ax_knob_suite.py in a child process with SPEQ_LIB_PATH pointing at it (one library per
process: the suite checks /proc/self/maps), against the CPU oracle. The default build is covered by the rest of the
GPU suite."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name -> the knobs it forces (kept in step with AXKNOB_* in the Makefile; checked below)
VARIANTS = {
    "kv1": "-DSPEQ_AX_SU=1 -DSPEQ_AX_SU_LOCAL=2 -DSPEQ_AX_REFILL=8 -DSPEQ_AX_BLOCKED=32 -DSPEQ_AX_P2_MARGIN=64 -DSPEQ_AX_PRIO_MIN=0 "
           "-DSPEQ_AX_WL=64 -DSPEQ_AX_MTILES=0",
    "kv2": "-DSPEQ_AX_WPB=2 -DSPEQ_AX_MIN_WAVES=4 -DSPEQ_AX_MIN_WAVES_LOCAL=3 -DSPEQ_AX_DEF_GLOBAL=192 "
           "-DSPEQ_AX_DEF_LOCAL=128",
    "kv3": "-DSPEQ_AX_SPEC_HW=1 -DSPEQ_AX_PRIO=0 -DSPEQ_AX_MPROOF=0",
}
KNOBS = {"SPEQ_AX_DEF_LOCAL", "SPEQ_AX_DEF_GLOBAL", "SPEQ_AX_WL", "SPEQ_AX_WPB", "SPEQ_AX_SU", "SPEQ_AX_SU_LOCAL",
         "SPEQ_AX_MIN_WAVES",
         "SPEQ_AX_MIN_WAVES_LOCAL", "SPEQ_AX_REFILL", "SPEQ_AX_BLOCKED", "SPEQ_AX_SPEC_HW", "SPEQ_AX_PRIO",
         "SPEQ_AX_PRIO_MIN", "SPEQ_AX_P2_MARGIN", "SPEQ_AX_MPROOF", "SPEQ_AX_MTILES"}


def test_variants_cover_every_knob():
    forced = {f.split("=")[0][2:] for v in VARIANTS.values() for f in v.split()}
    assert forced == KNOBS
    src = "".join(open(os.path.join(ROOT, "speq_amd", "csrc", f)).read() for f in ("ax_common.hpp", "ax_scan.hip"))
    import re
    defined = set(re.findall(r"#ifndef (SPEQ_AX_[A-Z0-9_]+)", src))
    assert defined == KNOBS, defined ^ KNOBS
    mk = open(os.path.join(ROOT, "Makefile")).read()
    for name, flags in VARIANTS.items():
        assert f"AXKNOB_{name} := {flags}" in mk, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_knob_variant_matches_oracle(name):
    lib = os.path.join(ROOT, "build", "axknobs", name, "libspeq_scan.so")
    assert os.path.exists(lib), f"{lib} missing: run `make axknobs` (build() does)"
    env = dict(os.environ, SPEQ_LIB_PATH=lib)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "ax_knob_suite.py")], env=env,
                       capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, (name, p.stdout[-2000:], p.stderr[-3000:])
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["cases"] >= 60 and out["lib"] == os.path.realpath(lib)
