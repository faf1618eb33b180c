"""CPU oracle for the encrypted-token path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this package.  It is the checker, never the thing measured or
shipped: ``reticulum_amd`` never imports it.

* ``token_oracle.c`` (via :mod:`oracle.ctoken`) — plain-C restatement,
  bit-exact with the golden vectors in ``tests/golden/token_vectors.json``.
* :mod:`oracle.cpuref` — pure-Python restatement with the reference's work
  shape (byte-matrix AES with a fresh key schedule per call, hashlib HMAC),
  used as the "reference pure-Python CPU path" baseline on the GPU box where
  the reference itself may not run.
"""
