"""On a node with the library and a gfx950 device the drop-in import takes
the HIP Token (the fallback side is
tests/test_dropin_fallback.py)."""
import pytest

pytestmark = pytest.mark.gpu


def test_dropin_import_takes_the_hip_token():
    import reticulum_amd as rt
    assert rt.available()
    from reticulum_amd.dropin import Token, hkdf
    assert Token is rt.Token and hkdf is rt.hkdf
    t = Token(Token.generate_key())
    msg = bytes(range(256)) * 2
    assert t.decrypt(t.encrypt(msg)) == msg
