"""The C-ABI library loads and exports every entry point declared in include/*.h (no GPU calls)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ottohip_\w+|otto_synth_\w+)\s*\(", src)))


def test_ottohip_exports_all_declared_symbols():
    import otto_recommender_amd._lib as L
    lib = L.load()
    names = _declared("ottohip.h")
    assert "ottohip_covis_count" in names and len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(L.SIGNATURES), set(names) ^ set(L.SIGNATURES)


def test_ottosynth_exports():
    lib = ctypes.CDLL(os.path.join(ROOT, "otto-recommender_amd", "libottosynth.so"))
    for n in _declared("ottosynth.h"):
        assert hasattr(lib, n), n


def test_library_is_gfx950_code_object():
    blob = open(os.path.join(ROOT, "otto-recommender_amd", "libottohip.so"), "rb").read()
    assert b"gfx950" in blob


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "otto-recommender_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", txt).lower() or f.endswith(".md"), f
