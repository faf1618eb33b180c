"""ctypes binding of librnstok.so (include/rnstok.h).

The HIP library is the only compute path: if it is missing or no gfx950
device is usable, every call raises :class:`NativeUnavailable` — there is no
CPU fallback.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# RNSTOK_LIB: an alternative build of the same library (A/B experiments, tools/)
LIB_PATH = os.environ.get("RNSTOK_LIB") or os.path.join(_HERE, "librnstok.so")

RT_OK, RT_E_INVAL, RT_E_HIP, RT_E_NOMEM, RT_E_NODEV = 0, -1, -2, -3, -4
RT_F_SORT_BY_LENGTH = 1
RT_ST_OK, RT_ST_TOO_SHORT, RT_ST_BAD_HMAC, RT_ST_BAD_CT_LEN, RT_ST_BAD_PAD = 0, 1, 2, 3, 4
RT_KERNEL_GENERAL, RT_KERNEL_ENC_LONG4, RT_KERNEL_ENC_LONG, RT_KERNEL_DEC_LONG2 = 0, 1, 2, 3
RT_KERNEL_ENC_SPLIT = 4
# the RNSTOK_ABI_VERSION (include/rnstok.h) these bindings are written for;
# load() refuses any other build of the library
ABI_VERSION = 2

# (name, restype, argtypes) for every entry point declared in include/rnstok.h
_vp, _u32, _u64, _i32, _int = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int
SIGNATURES = [
    ("rt_abi_version", _int, []),
    ("rt_last_error", ctypes.c_char_p, []),
    ("rt_device_count", _int, []),
    ("rt_create", _vp, [_int]),
    ("rt_destroy", None, [_vp]),
    ("rt_num_cus", _int, [_vp]),
    ("rt_keyset_create", _vp, [_vp, _vp, _u32, _u32]),
    ("rt_keyset_create_device", _vp, [_vp, _vp, _u32, _u32, _vp]),
    ("rt_keyset_destroy", None, [_vp]),
    ("rt_keyset_size", _u32, [_vp]),
    ("rt_token_len", _u64, [_u64]),
    ("rt_plan_uniform", _int, [_vp, _u32, _u32, _int, _int]),
    ("rt_encrypt_interleaved", _int, [_vp, _vp, _u32, _vp, _vp, _vp, _u32, _vp]),
    ("rt_decrypt_interleaved", _int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32, _vp]),
    ("rt_encrypt", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp]),
    ("rt_encrypt_uniform", _int, [_vp, _vp, _u64, _u32, _vp, _vp, _vp, _u64, _u32, _vp]),
    ("rt_decrypt", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp]),
    ("rt_decrypt_uniform", _int, [_vp, _vp, _u64, _u32, _vp, _vp, _u64, _vp, _vp, _u32, _vp]),
    ("rt_verify", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp]),
    ("rt_verify_host", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _u32]),
    ("rt_workspace_bytes", _u64, [_u32]),
    ("rt_encrypt_ex", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp]),
    ("rt_decrypt_ex", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp]),
    ("rt_encrypt_host", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32]),
    ("rt_decrypt_host", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32]),
    ("rt_hkdf", _int, [_vp, _vp, _u64, _u32, _vp, _u64, _u32, _vp, _u32, _vp, _u64, _u32, _u32, _vp]),
    ("rt_hkdf_host", _int, [_vp, _vp, _u64, _u32, _vp, _u64, _u32, _vp, _u32, _vp, _u64, _u32, _u32]),
    ("rt_keyset_create_hkdf", _vp, [_vp, _vp, _u64, _u32, _vp, _u64, _u32, _vp, _u32, _u32, _u32, _vp]),
    ("rt_verify_trials", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _vp]),
    ("rt_verify_trials_host", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32]),
    ("rt_map_hashes", _int, [_vp, _vp, _vp, _vp, _u64, _u32, _vp, _u32, _vp, _u32, _u32, _vp, _vp, _u32, _vp]),
    ("rt_resource_hashmap_host", _int, [_vp, _vp, _u64, _u32, _vp, _u32, _u32, _vp, _vp]),
    ("rt_hdlc_frame_workspace_bytes", _u64, [_u32]),
    ("rt_hdlc_frame", _int, [_vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp]),
    ("rt_hdlc_deframe_workspace_bytes", _u64, [_u64]),
    ("rt_hdlc_deframe", _int, [_vp, _vp, _u64, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _vp]),
    ("rt_hdlc_deframe_slots", _int, [_vp, _vp, _u64, _u32, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _vp]),
    ("rt_ifac_mask", _int, [_vp, _vp, _vp, _vp, _vp, _u32, _vp, _u32, _vp, _vp, _u32, _vp]),
    ("rt_ifac_unmask", _int, [_vp, _vp, _vp, _vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _u32, _vp]),
    ("rt_packet_unpack", _int, [_vp, _vp, _vp, _vp, _vp, _u32, _vp]),
    ("rt_frames_compact_workspace_bytes", _u64, [_u64]),
    ("rt_frames_compact", _int, [_vp, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("rt_token_spans", _int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    ("rt_packet_pack_headers", _int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp]),
    ("rt_device_alloc", _vp, [_vp, _u64]),
    ("rt_device_free", None, [_vp, _vp]),
    ("rt_host_alloc", _vp, [_u64]),
    ("rt_host_free", None, [_vp]),
    ("rt_memcpy_h2d", _int, [_vp, _vp, _vp, _u64, _vp]),
    ("rt_memcpy_d2h", _int, [_vp, _vp, _vp, _u64, _vp]),
    ("rt_memcpy_d2h_upto", _int, [_vp, _vp, _vp, _u64, _vp, _vp]),
    ("rt_stream_sync", _int, [_vp, _vp]),
    ("rt_clock_stamps", _int, [_vp, _vp]),
]


class NativeUnavailable(RuntimeError):
    """librnstok.so could not be loaded or no gfx950 device is usable."""


class NativeError(RuntimeError):
    """A librnstok call returned a negative RT_E_* code."""

    def __init__(self, code, msg):
        super().__init__(f"librnstok error {code}: {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()


def _share_hip_runtime_with_torch():
    """One HIP runtime per process.

    torch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7, loaded from
    torch/lib by name ``libamdhip64.so``); librnstok NEEDs libamdhip64.so.7.
    Loading librnstok first would pull /opt/rocm's copy and torch would then
    load a second runtime that finds no GPU.  When torch is installed, preload
    its copy globally so librnstok binds to it and torch later reuses it."""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return
    cand = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(cand):
        try:
            ctypes.CDLL(os.path.realpath(cand), mode=ctypes.RTLD_GLOBAL)
        except OSError:
            pass


def load():
    """Load librnstok.so and bind every declared symbol (no GPU needed)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeUnavailable(
                    f"{LIB_PATH} not found: build it with `make -C reticulum_amd/csrc` "
                    "(or __graft_entry__.build()); there is no CPU fallback")
            _share_hip_runtime_with_torch()
            try:
                lib = ctypes.CDLL(LIB_PATH)
            except OSError as e:
                raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
            missing = [name for name, _, _ in SIGNATURES if not hasattr(lib, name)]
            if missing:
                raise NativeUnavailable(f"{LIB_PATH} is older than these bindings (missing {', '.join(missing[:4])}"
                                        f"{' ...' if len(missing) > 4 else ''}): rebuild it")
            for name, res, args in SIGNATURES:
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            if lib.rt_abi_version() != ABI_VERSION:
                raise NativeUnavailable(f"{LIB_PATH} has ABI version {lib.rt_abi_version()}, these bindings expect "
                                        f"{ABI_VERSION}: rebuild it")
            _lib = lib
    return _lib


def last_error():
    msg = load().rt_last_error()
    return msg.decode(errors="replace") if msg else ""


def check(rc):
    if rc < 0:
        raise NativeError(rc, last_error())
    return rc


_contexts = {}


def context(device=None):
    """Process-wide context for ``device`` (default: $RNSTOK_DEVICE or 0)."""
    if device is None:
        device = int(os.environ.get("RNSTOK_DEVICE", "0"))
    ctx = _contexts.get(device)
    if ctx is None:
        lib = load()
        with _lock:
            ctx = _contexts.get(device)
            if ctx is None:
                ctx = lib.rt_create(device)
                if not ctx:
                    raise NativeUnavailable(f"rt_create({device}) failed: {last_error()}")
                _contexts[device] = ctx
    return ctx


def unavailable_reason(device=None):
    """None when librnstok.so loads and a gfx950 device answers rt_create,
    else why not (the message of the failure)."""
    try:
        context(device)
        return None
    except (NativeUnavailable, OSError, ValueError) as e:
        # OSError: the runtime itself fails to load; ValueError: a bad
        # RNSTOK_DEVICE value.  Either way the caller takes the reference path.
        return str(e)


def available(device=None):
    """True when librnstok.so loads and a gfx950 device answers rt_create.

    The drop-in import (``reticulum_amd.dropin``) checks this, so a node
    without the library or the GPU falls back to the reference's Token the
    way RNS/Cryptography/Provider.py:43-61 always leaves a working backend,
    instead of every Link.decrypt returning None (RNS/Link.py:1175-1182)."""
    return unavailable_reason(device) is None
