"""The documented drop-in swap falls back to the
reference's Token when the HIP library or a gfx950 device is unusable, the
way RNS/Cryptography/Provider.py:43-61 always leaves a working backend
(VERDICT r04 missing #4: otherwise Link.decrypt returns None for every
packet, RNS/Link.py:1175-1182).  Each case runs in a fresh interpreter, as a
node would import RNS.Cryptography."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

SWAP = """
import sys
sys.dont_write_bytecode = True
sys.path.insert(0, {root!r})
try:
    from reticulum_amd.dropin import Token
    which = "gpu"
except ImportError:
    sys.path.append({ref!r})
    from RNS.Cryptography import Token      # the reference's class (Cryptography/__init__.py:38)
    which = "reference"
t = Token(Token.generate_key())
assert t.decrypt(t.encrypt(b"hello")) == b"hello"
print(which, Token.__module__)
"""


def _run(env_extra):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", **env_extra)
    r = subprocess.run([sys.executable, "-c", SWAP.format(root=ROOT, ref=REF)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.split()


def _device_visible():
    from reticulum_amd import _native
    try:
        return _native.load().rt_device_count() > 0
    except _native.NativeUnavailable:
        return False


def test_dropin_import_fails_without_library():
    env = dict(os.environ, RNSTOK_LIB=os.path.join(ROOT, "no-such-librnstok.so"))
    r = subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r}); import reticulum_amd.dropin"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "ImportError" in r.stderr, r.stderr[-2000:]
    # the package itself still imports (its calls raise NativeUnavailable)
    r = subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r}); import reticulum_amd as rt; "
                        "print(rt.available())"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "False", r.stderr[-2000:]


@pytest.mark.reference
@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "RNS")), reason="reference checkout absent")
def test_swap_falls_back_to_reference_token_without_library():
    which, mod = _run({"RNSTOK_LIB": os.path.join(ROOT, "no-such-librnstok.so")})
    assert which == "reference" and mod == "RNS.Cryptography.Token"


@pytest.mark.reference
@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "RNS")), reason="reference checkout absent")
def test_swap_falls_back_to_reference_token_without_device():
    if _device_visible():
        pytest.skip("a GPU is visible: the swap takes the HIP Token (tests/test_dropin_gpu.py)")
    which, mod = _run({})
    assert which == "reference" and mod == "RNS.Cryptography.Token"


def _stub_library(tmp_path, drop=None, abi=None):
    """A stand-in librnstok.so built from the binding table: every entry point
    returns 0, `drop` is left out, rt_abi_version returns `abi`."""
    from reticulum_amd import _native
    lines = []
    for name, _, _ in _native.SIGNATURES:
        if name == drop:
            continue
        body = f"return {abi if abi is not None else _native.ABI_VERSION};" if name == "rt_abi_version" else "return 0;"
        lines.append(f"long {name}(void) {{ {body} }}")
    src = tmp_path / "stub.c"
    src.write_text("\n".join(lines) + "\n")
    so = tmp_path / "libstub.so"
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)])
    return str(so)


def _dropin_outcome(lib):
    env = dict(os.environ, RNSTOK_LIB=lib)
    code = (f"import sys; sys.path.insert(0, {ROOT!r})\n"
            "import reticulum_amd as rt\n"
            "print('available', rt.available())\n"
            "try:\n"
            "    import reticulum_amd.dropin\n"
            "    print('dropin imported')\n"
            "except ImportError as e:\n"
            "    print('ImportError', e)\n")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_dropin_import_fails_on_library_missing_a_symbol(tmp_path):
    """a library older than the bindings (one entry point absent)
    must read as unavailable, so the swap's `except ImportError` falls back,
    instead of an AttributeError escaping the import."""
    out = _dropin_outcome(_stub_library(tmp_path, drop="rt_clock_stamps"))
    assert "available False" in out and "ImportError" in out and "older than these bindings" in out, out


def test_dropin_import_fails_on_abi_version_mismatch(tmp_path):
    out = _dropin_outcome(_stub_library(tmp_path, abi=1))
    assert "available False" in out and "ImportError" in out and "ABI version 1" in out, out


def test_available_false_on_bad_device_value():
    env = dict(os.environ, RNSTOK_DEVICE="not-a-number")
    r = subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r}); import reticulum_amd as rt; "
                        "print(rt.available())"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "False", r.stderr[-2000:]
