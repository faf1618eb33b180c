"""The C-ABI library loads without a GPU and exports every entry point that
include/rnstok.h declares, with the declared Python binding; without a device
the product path fails loudly (no CPU fallback)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "rnstok.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from reticulum_amd import _native
    bound = sorted(name for name, _, _ in _native.SIGNATURES)
    assert bound == declared_functions()


def test_library_exports_every_declared_symbol():
    from reticulum_amd import _native
    lib = _native.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.rt_abi_version() == _native.ABI_VERSION
    assert lib.rt_token_len(500) == 560
    assert lib.rt_token_len(0) == 64
    assert lib.rt_token_len(16384) == 16448


def test_library_targets_gfx950_only():
    """The offload bundle inside librnstok.so holds a gfx950 code object and
    no other GPU target."""
    from reticulum_amd import _native
    with open(_native.LIB_PATH, "rb") as f:
        blob = f.read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_no_device_fails_loudly():
    from reticulum_amd import _native
    import reticulum_amd as rt
    lib = _native.load()
    if lib.rt_device_count() > 0:
        pytest.skip("a GPU is visible; covered by -m gpu tests")
    with pytest.raises(rt.NativeUnavailable):
        _native.context(0)
    with pytest.raises(rt.NativeUnavailable):
        rt.Token(bytes(64)).encrypt(b"x")


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "reticulum_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "from oracle" not in text, f
                assert "liboracle" not in text, f
