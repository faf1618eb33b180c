"""Group commit for per-packet Token calls from many threads.

Reticulum calls ``Token`` one packet at a time and synchronously: every
interface's reader thread decrypts the packets it hands to Transport
(``RNS/Interfaces/TCPInterface.py:175,294`` -> ``Transport.inbound`` ->
``Link.receive`` -> ``Link.decrypt``, ``RNS/Link.py:1175-1182``), and
application, Resource and Channel threads encrypt (``RNS/Link.py:1161-1173``,
``RNS/Identity.py:829-830``).  Each such call through ``reticulum_amd.Token``
is one GPU round trip (≈50-65 µs at 500 B), so a node with
many busy interfaces is bound by round trips, not by the kernels.

``CoalescingToken`` has ``Token``'s surface and semantics but hands its calls
to a process-wide ``Coalescer``, which runs them as group commits: the first
caller to arrive becomes the leader and runs every call queued at that moment
as one batch (one ``rt_encrypt_host`` / ``rt_decrypt_host`` /
``rt_verify_host`` per operation and key length, the batch's distinct keys in
one key set indexed per packet), while the calls that arrive during it queue
for the next leader.  An uncontended call is its own batch of one (no timer,
no helper thread, no added latency); under contention the batch grows with
the number of waiting threads.  Results and exceptions are per call and equal
to ``Token``'s (the same status-to-message mapping, ``Token.py:77-114``).
"""
import os
import threading

import numpy as np

from .token import AES, KeySet, Packed, RT_ST_OK, Token, status_message

_ENC, _DEC, _VER = 0, 1, 2


class _Call:
    __slots__ = ("op", "key", "data", "result", "error", "done")

    def __init__(self, op, key, data):
        self.op, self.key, self.data = op, key, data
        self.result = self.error = None
        self.done = False


class Coalescer:
    """Group-commit executor for Token calls on one device (see module doc).

    ``max_batch`` bounds one leader's batch; ``stats`` counts calls and
    batches (calls / batches is the mean batch size)."""

    def __init__(self, device=None, max_batch=16384):
        self.device = device
        self.max_batch = max_batch
        self._cv = threading.Condition(threading.Lock())
        self._queue = []
        self._leader = False
        self.stats = {"calls": 0, "batches": 0}

    def run(self, op, key, data):
        c = _Call(op, key, data)
        with self._cv:
            self._queue.append(c)
            # a call queued while another leader's batch runs waits for that
            # batch to end; if it was not in it, its thread leads the next one
            while self._leader and not c.done:
                self._cv.wait()
            if not c.done:
                self._leader = True
                batch = self._queue[:self.max_batch]
                del self._queue[:len(batch)]
        if not c.done:
            try:
                self._execute(batch)
            finally:
                with self._cv:
                    for b in batch:
                        b.done = True
                    self._leader = False
                    self.stats["calls"] += len(batch)
                    self.stats["batches"] += 1
                    self._cv.notify_all()
        if c.error is not None:
            raise c.error
        return c.result

    def _execute(self, batch):
        groups = {}
        for c in batch:
            groups.setdefault((c.op, len(c.key)), []).append(c)
        for (op, _), calls in groups.items():
            try:
                self._run_group(op, calls)
            except Exception as exc:             # a library error fails the group's calls, not the leader
                for c in calls:
                    c.error = exc

    def _run_group(self, op, calls):
        index, keys = {}, []
        for c in calls:
            if c.key not in index:
                index[c.key] = len(keys)
                keys.append(c.key)
        ks = KeySet(keys, device=self.device)
        kidx = np.fromiter((index[c.key] for c in calls), dtype=np.uint32, count=len(calls))
        data = Packed.from_list([c.data for c in calls])
        if op == _ENC:
            out = ks.encrypt_batch(data, ivs=np.frombuffer(os.urandom(16 * len(calls)), np.uint8),
                                   key_idx=kidx)                   # fresh IVs, Token.py:89
            for i, c in enumerate(calls):
                c.result = out[i]
        elif op == _DEC:
            out, status, detail = ks._decrypt_raw(data, key_idx=kidx)
            for i, c in enumerate(calls):
                if status[i] == RT_ST_OK:
                    c.result = out[i]
                else:
                    c.error = ValueError(status_message(int(status[i]), len(c.data), int(detail[i])))
        else:
            status = ks.verify_batch(data, key_idx=kidx)
            for i, c in enumerate(calls):
                c.result = bool(status[i] == RT_ST_OK)


_coalescers = {}
_coalescers_lock = threading.Lock()


def coalescer(device=None):
    """The process-wide Coalescer of ``device``."""
    with _coalescers_lock:
        c = _coalescers.get(device)
        if c is None:
            c = _coalescers[device] = Coalescer(device)
        return c


class CoalescingToken(Token):
    """``Token`` whose calls are group-committed with other threads' calls
    (see module doc).  Same constructor, errors and results as ``Token``
    (``Token.py:40-114``); batch extensions as ``Token``."""

    def __init__(self, key=None, mode=AES, device=None):
        super().__init__(key, mode=mode, device=device)
        self._coalescer = coalescer(device)

    def verify_hmac(self, token):                               # Token.py:77-84
        if len(token) <= 32:
            raise ValueError("Cannot verify HMAC on token of only " + str(len(token)) + " bytes")
        return self._coalescer.run(_VER, self._key, bytes(token))

    def encrypt(self, data=None):                               # Token.py:87-97
        if not isinstance(data, bytes):
            raise TypeError("Token plaintext input must be bytes")
        return self._coalescer.run(_ENC, self._key, data)

    def decrypt(self, token=None):                              # Token.py:100-114
        if not isinstance(token, bytes):
            raise TypeError("Token must be bytes")
        if len(token) <= 32:
            raise ValueError("Cannot verify HMAC on token of only " + str(len(token)) + " bytes")
        return self._coalescer.run(_DEC, self._key, token)
