"""The drop-in import for the reference's crypto package.

``import reticulum_amd.dropin`` raises ImportError unless librnstok.so loads
and a gfx950 device answers (``reticulum_amd.available()``), so the one-line
swap INTEGRATION.md §1 gives for ``RNS/Cryptography/__init__.py:38``

    try:
        from reticulum_amd.dropin import Token
    except ImportError:
        from .Token import Token

keeps a working Token on every node, as the reference's backend selection
does (RNS/Cryptography/Provider.py:43-61).  Importing ``reticulum_amd``
itself never fails: its calls raise NativeUnavailable where the library or
the device is missing (the batch API and the tests rely on that).
"""
from ._native import unavailable_reason as _unavailable_reason

_why = _unavailable_reason()
if _why is not None:
    raise ImportError("reticulum_amd: librnstok.so or a gfx950 device is unavailable (%s); "
                      "use the reference implementation" % _why)

from .hkdf import hkdf  # noqa: E402,F401
from .token import AES, AES_128_CBC, AES_256_CBC, Token, TOKEN_OVERHEAD  # noqa: E402,F401
