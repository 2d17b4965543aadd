"""Dynamic-LDS limits are raised once, from one registry (csrc/common.h, csrc/devmem.cpp:
fa_lds_prepare), never on a launch path: the round-3 profiled crash had eight host threads racing
through per-site hipFuncSetAttribute calls."""
import glob
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fairify_amd", "csrc")


def test_no_attribute_calls_on_launch_paths():
    hits = []
    for path in glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")):
        src = open(path).read()
        for m in re.finditer(r"hipFuncSetAttribute\s*\(", src):
            hits.append(os.path.basename(path))
    assert hits == ["devmem.cpp"], hits           # only fa_lds_prepare


def test_every_checked_launch_file_registers_its_kernels():
    for path in glob.glob(os.path.join(CSRC, "*.hip")):
        src = open(path).read()
        if "fa_lds_ok(" in src:
            assert "FA_LDS_REGISTER(" in src, os.path.basename(path)


def test_registry_populated_at_load():
    try:
        import fairify_amd._C as C
    except ImportError:
        import pytest

        pytest.skip("extension not built")
    assert C.lds_registered() >= 40
