"""Drop-in proof: the reference's own callers run unchanged on reticulum_amd.Token.

Build container only (needs the reference checkout at /root/reference; it is
skipped elsewhere and never travels to the GPU box).  The reference's
``Token`` class is swapped for ``reticulum_amd.Token`` in every module that
imported it (RNS/Identity.py:42, RNS/Link.py:32, RNS/Destination.py:37), then
the reference's own token KAT (tests/identity.py:148-158) and its random
Identity.encrypt/decrypt round trips (tests/identity.py:160-194, fewer
iterations) run through the swapped class.  On CPU the HIP library is stood in
for by tests/fake_native.py; the GPU suite runs the same class on the kernels.
"""
import os
import sys

import pytest

REF = "/root/reference"
pytestmark = [pytest.mark.reference,
              pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "RNS")), reason="reference checkout absent")]


@pytest.fixture(scope="module")
def RNS():
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.append(REF)
    import RNS as rns  # noqa: N811
    return rns


@pytest.fixture
def swapped(RNS, monkeypatch):
    import fake_native
    import reticulum_amd
    fake = fake_native.install(monkeypatch)
    ref_token = sys.modules["RNS.Cryptography.Token"].Token
    for mod in ("RNS.Identity", "RNS.Link", "RNS.Destination"):
        monkeypatch.setattr(sys.modules[mod], "Token", reticulum_amd.Token)
    return fake, ref_token


def _literal(name):
    src = open(os.path.join(REF, "tests", "identity.py")).read()
    for line in src.splitlines():
        if line.strip().startswith(name + " ="):
            return line.split("=", 1)[1].strip().strip('"')
    raise KeyError(name)


def test_identity_kat_through_swapped_token(RNS, swapped):
    fake, _ = swapped
    key0 = open(os.path.join(REF, "tests", "identity.py")).read().split('fixed_keys = [')[1].split('("')[1].split('"')[0]
    fid = RNS.Identity.from_bytes(bytes.fromhex(key0))
    pt = fid.decrypt(bytes.fromhex(_literal("fixed_token")))
    assert pt == bytes.fromhex(_literal("encrypted_message"))
    assert ("decrypt", 1) in fake.calls           # went through reticulum_amd.Token


def test_identity_round_trips_through_swapped_token(RNS, swapped):
    fake, _ = swapped
    for i in range(1, 13):
        mlen = i % (RNS.Reticulum.MTU // 2) + (RNS.Reticulum.MTU // 2)
        msg = os.urandom(mlen)
        id1 = RNS.Identity()
        id2 = RNS.Identity(create_keys=False)
        id2.load_public_key(id1.get_public_key())
        token = id2.encrypt(msg)
        assert id1.decrypt(token) == msg
    assert sum(1 for c in fake.calls if c[0] == "encrypt") >= 12


def test_cross_compat_with_reference_token(RNS, swapped):
    import reticulum_amd
    _, RefToken = swapped
    key = os.urandom(64)
    ours, ref = reticulum_amd.Token(key), RefToken(key)
    for L in (0, 1, 15, 16, 100, 431):
        msg = os.urandom(L)
        assert ref.decrypt(ours.encrypt(msg)) == msg
        assert ours.decrypt(ref.encrypt(msg)) == msg


def test_group_destination_keys(RNS, swapped):
    """GROUP destinations hold a Token built from Token.generate_key()
    (RNS/Destination.py:544-558)."""
    import reticulum_amd
    key = reticulum_amd.Token.generate_key()
    t = reticulum_amd.Token(key)
    assert t.decrypt(t.encrypt(b"group payload")) == b"group payload"
