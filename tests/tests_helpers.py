"""Small helpers shared by the test modules."""


def b(h):
    return bytes.fromhex(h)
