"""CPU-side checks of the boundary: the C-ABI library loads and exports every symbol that
include/pbccs_amd.h declares (no compute calls: there is no GPU here), and host helpers behave."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "pbccs_amd.h")).read()
    return sorted(set(re.findall(r"\b(pbccs_[a-z_]+)\s*\(", hdr)))


def test_header_declarations_have_bindings():
    from pbccs_amd import lib
    assert set(_declared_symbols()) == set(lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    from pbccs_amd import lib
    if not os.path.exists(lib.LIB_PATH):
        pytest.skip("libpbccs_amd.so not built (run __graft_entry__.build())")
    L = lib.load()
    for name in _declared_symbols():
        assert hasattr(L, name), name


def test_engine_create_fails_loudly_without_device():
    import pbccs_amd
    from pbccs_amd import lib
    if not os.path.exists(lib.LIB_PATH):
        pytest.skip("library not built")
    if lib.load().pbccs_device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(pbccs_amd.PbccsError):
        pbccs_amd.Engine(0)


def test_synthetic_generator_is_deterministic():
    from pbccs_amd import synth
    a = synth.make_zmws(2, 300, 3, seed=9)
    b = synth.make_zmws(2, 300, 3, seed=9)
    assert a == b
    for z in a:
        assert set(z["draft"]) <= set("ACGT")
        assert all(r["te"] == len(z["draft"]) for r in z["reads"])
        assert [r["strand"] for r in z["reads"]] == [0, 1, 0]
