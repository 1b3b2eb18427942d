"""Python host mirror of the reference ``SphereflakeRaytracer::Sphereflake`` class
(/root/reference/sphereflake/Sphereflake.h:13-58) over the gfx950 C ABI
(include/sphereflake/sf.h, built as build/libsphereflake_hip.so).

There is no CPU fallback: if the HIP library is missing or the device is not a gfx950,
constructing a :class:`Sphereflake` raises. The CPU restatement under ``oracle/`` is test
infrastructure and is never imported from here.

Names follow the reference: ``SetView``, ``GetGBuffer``, ``GetMaxDepthReached``,
``ResetMaxDepthReached``, ``GetRaysPerSecond``, ``ResetRaysPerSecond``,
``GetClosestSphereDistance``, ``ResetClosestSphereDistance``, ``Initialize`` (frame-less
progressive mode), plus ``Render`` (one deterministic full frame). ``Camera`` mirrors
reference camera.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from dataclasses import dataclass

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)                 # sphereflake-raytracer_amd/
# SF_LIB selects another build of the same library (e.g. the stamp diagnostics build_phases/)
LIB_PATH = os.environ.get("SF_LIB") or os.path.join(ROOT_DIR, "build", "libsphereflake_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(ROOT_DIR), "include", "sphereflake", "sf.h")

SF_OK, SF_EINVAL, SF_ENOMEM, SF_EHIP, SF_ENODEV, SF_ENOVIEW, SF_EDEPTH, SF_ESTATE = 0, -1, -2, -3, -4, -5, -6, -7
SF_KERNEL_WAVE, SF_KERNEL_PER_RAY = 0, 1
SF_MAX_DEPTH_LIMIT = 31
FLT_MAX = float(np.finfo(np.float32).max)

# Camera of reference main.cpp:92-96; BASELINE configs scale the position by K.
DEFAULT_CAMERA_POSITION = (-5.4098, -7.2139, 1.19006)
DEFAULT_PITCH = -1.371
DEFAULT_YAW = 0.921999
SF_DIAG_WAVES = 65536            # per-wave diagnostic records (sf_internal.h)


class SphereflakeError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _strerror(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


class sf_render_params(ctypes.Structure):
    _fields_ = [("band_rows", ctypes.c_uint32), ("band_count", ctypes.c_uint32),
                ("band_index", ctypes.c_uint32), ("compact", ctypes.c_uint32),
                ("kernel", ctypes.c_uint32), ("emit_aux", ctypes.c_uint32),
                ("max_depth", ctypes.c_uint32), ("packed", ctypes.c_uint32),
                ("stream", ctypes.c_void_p)]


class sf_stats(ctypes.Structure):
    _fields_ = [("max_depth", ctypes.c_int32), ("closest", ctypes.c_float),
                ("rays", ctypes.c_int64), ("overflow_tiles", ctypes.c_int64)]


class sf_post_params(ctypes.Structure):
    _fields_ = [("sample_radius", ctypes.c_float), ("intensity", ctypes.c_float), ("scale", ctypes.c_float),
                ("bias", ctypes.c_float), ("normal_threshold", ctypes.c_float), ("depth_threshold", ctypes.c_float),
                ("camera_position", ctypes.c_float * 3), ("downscale", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("stream", ctypes.c_void_p)]


SF_VARIANT_AVX = 0
SF_VARIANT_SSE = 1
SF_POST_GENERAL = 1
SF_POST_UNIT_NORMALS = 2
SF_DUMP_IMAGE, SF_DUMP_NORMALS, SF_DUMP_POSITIONS_PFM, SF_DUMP_NORMALS_PFM = 0, 1, 2, 3

# exported symbol -> (restype, argtypes); checked against include/sphereflake/sf.h by the tests
_F = ctypes.POINTER(ctypes.c_float)
_U = ctypes.POINTER(ctypes.c_uint32)
_CTX = ctypes.c_void_p
SIGNATURES = {
    "sf_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "sf_destroy": (None, [_CTX]),
    "sf_set_view": (ctypes.c_int, [_CTX, _F, _F, _F, _F]),
    "sf_set_setup": (ctypes.c_int, [_CTX, _F, _F]),
    "sf_get_setup": (ctypes.c_int, [_CTX, _F, _F]),
    "sf_render": (ctypes.c_int, [_CTX, ctypes.POINTER(sf_render_params)]),
    "sf_render_to": (ctypes.c_int, [_CTX, ctypes.POINTER(sf_render_params), ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p]),
    "sf_render_frames": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                        ctypes.POINTER(sf_render_params)]),
    "sf_slab_rows": (ctypes.c_uint32, [ctypes.c_uint32] * 4),
    "sf_unpack_bands": (ctypes.c_int, [_CTX, ctypes.c_void_p] + [ctypes.c_uint32] * 5 + [ctypes.c_void_p]),
    "sf_unpack_slabs": (ctypes.c_int, [_CTX, ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [ctypes.c_void_p]),
    "sf_slab_bytes": (ctypes.c_uint32, [_CTX]),
    "sf_download": (ctypes.c_int, [_CTX, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "sf_download_async": (ctypes.c_int, [_CTX, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "sf_set_variant": (ctypes.c_int, [_CTX, ctypes.c_int]),
    "sf_get_variant": (ctypes.c_int, [_CTX]),
    "sf_lod_threshold": (ctypes.c_int, [ctypes.c_float, ctypes.c_float, _F]),
    "sf_division_by_reciprocal_exact": (ctypes.c_int, [ctypes.c_uint32]),
    "sf_post_defaults": (ctypes.c_int, [_CTX, ctypes.POINTER(sf_post_params)]),
    "sf_post_process": (ctypes.c_int, [_CTX, ctypes.POINTER(sf_post_params), ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "sf_download_image": (ctypes.c_int, [_CTX, ctypes.c_void_p]),
    "sf_ssao_noise": (ctypes.c_int, [_F]),
    "sf_save_image": (ctypes.c_int, [_CTX, ctypes.c_char_p, ctypes.c_int]),
    "sf_write_ppm": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]),
    "sf_write_pfm": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]),
    "sf_get_size": (ctypes.c_int, [_CTX, _U, _U]),
    "sf_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "sf_host_unregister": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_device_buffers": (ctypes.c_int, [_CTX] + [ctypes.POINTER(ctypes.c_void_p)] * 4),
    "sf_synchronize": (ctypes.c_int, [_CTX]),
    "sf_get_stats": (ctypes.c_int, [_CTX, ctypes.POINTER(sf_stats)]),
    "sf_reset_max_depth": (ctypes.c_int, [_CTX]),
    "sf_reset_rays": (ctypes.c_int, [_CTX]),
    "sf_reset_closest": (ctypes.c_int, [_CTX]),
    "sf_progressive": (ctypes.c_int, [_CTX, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]),
    "sf_camera_corners": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, _F, ctypes.c_float, ctypes.c_float,
                                         ctypes.c_float, ctypes.c_float, _F, _F, _F, _F]),
    "sf_child_transforms": (ctypes.c_int, [_F]),
    "sf_root_transform": (ctypes.c_int, [_F, _F]),
    "sf_depth_constants": (ctypes.c_int, [ctypes.c_uint32, _F, _F]),
    "sf_rsqrtps": (ctypes.c_float, [ctypes.c_float]),
    "sf_mt19937_jump": (ctypes.c_int, [_U, ctypes.c_uint64, _U]),
    "sf_set_tile_trace": (ctypes.c_int, [_CTX, ctypes.c_int]),
    "sf_get_tile_trace": (ctypes.c_int, [_CTX, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]),
    "sf_get_tile_order": (ctypes.c_int, [_CTX, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.c_size_t]),
    "sf_set_kernel_timing": (ctypes.c_int, [_CTX, ctypes.c_int]),
    "sf_kernel_times": (ctypes.c_int, [_CTX, _F, ctypes.c_uint32]),
    "sf_kernel_clocks": (ctypes.c_int, [_CTX, _F, ctypes.c_uint32]),
    "sf_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "sf_last_hip_error": (ctypes.c_int, [_CTX]),
    "sf_abi_version": (ctypes.c_int, []),
    "sf_build_id": (ctypes.c_char_p, []),
    "sf_device_count": (ctypes.c_int, []),
    "sf_context_stream": (ctypes.c_void_p, [_CTX]),
    "sf_group_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    "sf_group_destroy": (None, [ctypes.c_void_p]),
    "sf_group_size": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_group_member": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int]),
    "sf_group_set_view": (ctypes.c_int, [ctypes.c_void_p, _F, _F, _F, _F]),
    "sf_group_set_variant": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "sf_group_render": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "sf_group_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_group_download": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "sf_group_get_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(sf_stats)]),
    "sf_group_last_hip_error": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_group_reset_stats": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_group_slab_bytes": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_dist_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_dist_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "sf_dist_destroy": (None, [ctypes.c_void_p]),
    "sf_dist_slots": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_dist_context": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int]),
    "sf_dist_last_slot": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_dist_set_view": (ctypes.c_int, [ctypes.c_void_p, _F, _F, _F, _F]),
    "sf_dist_render": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_dist_render_bands": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_dist_render_bands_frames": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, _F]),
    "sf_dist_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_dist_download": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "sf_dist_get_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(sf_stats)]),
    "sf_dist_reset_stats": (ctypes.c_int, [ctypes.c_void_p]),
    "sf_dist_last_error": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "sf_dist_comm_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int] + [ctypes.POINTER(ctypes.c_int)] * 3),
    "sf_dist_slab_bytes": (ctypes.c_int, [ctypes.c_void_p]),
}
SF_ECOMM = -8
SF_DIST_ID_BYTES = 128

_lib = None
_lock = threading.Lock()


def build(force: bool = False) -> str:
    """Compile the gfx950 library in-tree (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", ROOT_DIR, "all"])
    return LIB_PATH


def lib() -> ctypes.CDLL:
    """Load build/libsphereflake_hip.so; raises if it is missing (no fallback path exists)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(f"HIP renderer library not built: {LIB_PATH} (run make -C {ROOT_DIR})")
            # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (SONAME
            # libamdhip64.so.7). Loading it first makes our NEEDED libamdhip64.so.7 resolve to the
            # same runtime, so torch tensors / streams and our contexts can be mixed freely.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            L = ctypes.CDLL(LIB_PATH)
            # (SF_LIB_PARTIAL=1: an older build under A/B -- entry points it predates are left unbound)
            partial = os.environ.get("SF_LIB_PARTIAL") == "1"
            for name, (res, args) in SIGNATURES.items():
                if partial and not hasattr(L, name):
                    continue
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def build_info() -> dict:
    """Which build is loaded: the source hash the library embeds (sf_build_id), the hash of the sources in
    this tree (scripts/source_hash.py), whether they agree, and the SHA-256 of the library file itself."""
    import hashlib
    import importlib.util
    with open(LIB_PATH, "rb") as f:
        lib_sha = hashlib.sha256(f.read()).hexdigest()[:16]
    embedded = lib().sf_build_id().decode()
    tree = None
    sh = os.path.join(os.path.dirname(ROOT_DIR), "scripts", "source_hash.py")
    if os.path.exists(sh):
        spec = importlib.util.spec_from_file_location("_sf_source_hash", sh)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        tree = m.source_hash()
    return {"source_sha256": embedded, "tree_source_sha256": tree, "lib_matches_tree": embedded == tree,
            "lib_sha256": lib_sha}


def _strerror(code: int) -> str:
    try:
        return lib().sf_strerror(code).decode()
    except Exception:  # library not loadable: still give a message
        return f"sphereflake error {code}"


def _check(rc: int, what: str = "", ctx=None) -> None:
    if rc != SF_OK:
        err = SphereflakeError(rc, what)
        if ctx is not None and rc == SF_EHIP:
            err.hip_error = lib().sf_last_hip_error(ctx)
        raise err


def _f32(a, n=None) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    if n is not None and a.size != n:
        raise ValueError(f"expected {n} floats, got {a.size}")
    return a


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_F)


_F3 = ctypes.c_float * 3


def _vec3(v):
    """A view vector as a ctypes float[3] (the per-frame SetView path: a tuple or list of 3 numbers is converted
    without numpy, ~6 us less host time per frame; float32 rounding as np.float32)."""
    if isinstance(v, (tuple, list)) and len(v) == 3:
        return _F3(*v)
    if isinstance(v, np.ndarray) and v.dtype == np.float32 and v.shape == (3,):
        return _F3(*v.tolist())
    return _F3(*_f32(v, 3).ravel().tolist())


# ----------------------------------------------------------------------------- host setup helpers

def child_transforms() -> np.ndarray:
    """9 unit child frames (reference Sphereflake.cpp:216-249), [9, 16] glm column-major."""
    out = np.zeros((9, 16), np.float32)
    _check(lib().sf_child_transforms(_fp(out)), "sf_child_transforms")
    return out


def root_transform(origin) -> np.ndarray:
    """Root transform of SetView (Sphereflake.cpp:83) for a ray origin, [16]."""
    o = _f32(origin, 3)
    out = np.zeros(16, np.float32)
    _check(lib().sf_root_transform(_fp(o), _fp(out)), "sf_root_transform")
    return out


def depth_constants(depth: int):
    """(radius r_d, exact LOD threshold T_d) used by the kernels at a depth."""
    r, t = ctypes.c_float(), ctypes.c_float()
    _check(lib().sf_depth_constants(depth, ctypes.byref(r), ctypes.byref(t)), "sf_depth_constants")
    return r.value, t.value


def lod_threshold(r: float, lod_constant: float = 70.0) -> float:
    """Exact T with sqrtf(t / r) < lod_constant || t < 0  <=>  t < T (Sphereflake.h:129,146)."""
    t = ctypes.c_float()
    _check(lib().sf_lod_threshold(ctypes.c_float(r), ctypes.c_float(lod_constant), ctypes.byref(t)),
           "sf_lod_threshold")
    return t.value


def rsqrtps(x: float) -> float:
    """x86 rsqrtps as reproduced by the renderer (host copy of the kernels' table)."""
    return lib().sf_rsqrtps(float(x))


def device_count() -> int:
    return lib().sf_device_count()


class Camera:
    """Mirror of reference camera.h (SphereflakeRaytracer::Camera): FOV 60, angles in radians."""

    def __init__(self, width: int, height: int):
        self.width, self.height = int(width), int(height)
        self.position = np.zeros(3, np.float32)
        self.fov, self.roll, self.pitch, self.yaw = 60.0, 0.0, 0.0, 0.0

    def SetPosition(self, p):
        self.position = _f32(p, 3).copy()

    def GetPosition(self):
        return self.position.copy()

    def SetPitch(self, v): self.pitch = float(v)
    def SetYaw(self, v): self.yaw = float(v)
    def SetRoll(self, v): self.roll = float(v)
    def SetFOV(self, v): self.fov = float(v)

    def corners(self):
        o, tl, tr, bl = (np.zeros(3, np.float32) for _ in range(4))
        pos = _f32(self.position, 3)
        _check(lib().sf_camera_corners(self.width, self.height, _fp(pos), self.pitch, self.yaw, self.roll,
                                       self.fov, _fp(o), _fp(tl), _fp(tr), _fp(bl)), "sf_camera_corners")
        return o, tl, tr, bl

    def GetTopLeft(self): return self.corners()[1]
    def GetTopRight(self): return self.corners()[2]
    def GetBottomLeft(self): return self.corners()[3]


def config_camera(width: int, height: int, K: float) -> Camera:
    """The fixed camera of the BASELINE configs: main.cpp:92-96 with position scaled by K."""
    cam = Camera(width, height)
    cam.SetPosition(np.asarray(DEFAULT_CAMERA_POSITION, np.float32) * np.float32(K))
    cam.SetPitch(np.float32(DEFAULT_PITCH))
    cam.SetYaw(np.float32(DEFAULT_YAW))
    cam.SetRoll(0.0)
    return cam


# ----------------------------------------------------------------------------- the renderer

@dataclass
class GBuffer:
    """Reference GBuffer (Sphereflake.h:7-11): positions / normals as [H, W, 4] float32 (x, y, z, 1)."""
    positions: np.ndarray
    normals: np.ndarray


SF_PACKED_NORMAL = 1   # band slab: float4 (nx, ny, nz, minT) per pixel, 16 B
SF_PACKED_INDEX = 2    # band slab: uint32 hit index per pixel, 4 B (where slab_bytes() == 4)


def render_params(band_rows=0, band_count=1, band_index=0, compact=False, kernel=SF_KERNEL_WAVE,
                  emit_aux=False, max_depth=0, stream=None, packed=0) -> sf_render_params:
    """packed: 0 / False (G-buffer layout), 1 / True (16 B slab), 2 (4 B hit-index slab)."""
    return sf_render_params(band_rows, band_count, band_index, int(bool(compact)), kernel, int(bool(emit_aux)),
                            max_depth, int(packed), stream)


class _FifoLock:
    """Ticket lock: waiters are served in arrival order (the C++ class's FairMutex, Sphereflake.hpp). The
    frame-less loop re-locks right after each batch; with a plain Lock a caller's SetView / GetGBuffer
    could lose to it for many batches in a row."""

    def __init__(self):
        self._c = threading.Condition(threading.Lock())
        self._next = 0
        self._serving = 0

    def __enter__(self):
        with self._c:
            t = self._next
            self._next += 1
            while self._serving != t:
                self._c.wait()
        return self

    def __exit__(self, *exc):
        with self._c:
            self._serving += 1
            self._c.notify_all()


def _views12(views) -> np.ndarray:
    """[(origin, top-left, top-right, bottom-left), ...] (or an n x 12 float32 array) -> a contiguous float32 n x 12
    array."""
    if isinstance(views, np.ndarray) and views.dtype == np.float32 and views.ndim == 2 and views.shape[1] == 12 \
            and views.flags.c_contiguous:
        return views
    return np.ascontiguousarray(np.array([[c for v in view for c in v] for view in views], np.float32).reshape(-1, 12))


def render_frames(flakes, **kw):
    """Each flake's current view into its own G-buffer, in ONE multi-frame persistent launch (sf_render_frames):
    bit for bit what flake.Render(**kw) does for each (whole frames or bands at frame positions)."""
    import contextlib
    p = render_params(**kw)
    arr = (ctypes.c_void_p * len(flakes))(*[f.ctx for f in flakes])
    with contextlib.ExitStack() as held:   # (every context's lock once, as each Render would take its own; a
        seen = set()                        # context given twice is the C ABI's SF_EINVAL, not a deadlock here)
        for f in flakes:
            if id(f) not in seen:
                seen.add(id(f))
                held.enter_context(f._mutex)
        _check(lib().sf_render_frames(arr, len(flakes), ctypes.byref(p)), "sf_render_frames", flakes[0].ctx)


class Sphereflake:
    """Drop-in for the reference class. Owns a device context (G-buffer in HBM)."""

    def __init__(self, width: int, height: int, device: int = 0):
        self.width, self.height, self.device = int(width), int(height), int(device)
        L = lib()
        h = ctypes.c_void_p()
        _check(L.sf_create(self.device, self.width, self.height, ctypes.byref(h)), "sf_create")
        self._ctx = h
        self._worker = None
        self._stop = threading.Event()
        self._mutex = _FifoLock()
        self._seed = 0
        self._counter = 0
        self._view_change = 0
        self._worker_error = None

    # lifetime --------------------------------------------------------------
    def close(self):
        self.release_pinned()
        self._stop.set()
        if self._worker is not None:
            self._worker.join()
            self._worker = None
        if getattr(self, "_ctx", None):
            lib().sf_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def ctx(self):
        return self._ctx

    # view ------------------------------------------------------------------
    def SetView(self, origin, topLeft, topRight, bottomLeft):
        o, tl, tr, bl = (_vec3(v) for v in (origin, topLeft, topRight, bottomLeft))
        with self._mutex:   # (the frame-less loop's batches read the view)
            _check(lib().sf_set_view(self._ctx, o, tl, tr, bl), "SetView", self._ctx)
            self._view_change = self._counter

    def GetViewChangePacket(self) -> int:
        """The frame-less loop's packet counter when the last SetView took effect (batches from it on trace
        the new view)."""
        with self._mutex:
            return self._view_change

    def SetCamera(self, cam: Camera):
        o, tl, tr, bl = cam.corners()
        self.SetView(o, tl, tr, bl)

    def SetSetup(self, child, root):
        c, r = _f32(child, 144), _f32(root, 16)
        _check(lib().sf_set_setup(self._ctx, _fp(c), _fp(r)), "sf_set_setup", self._ctx)

    def GetSetup(self):
        c, r = np.zeros((9, 16), np.float32), np.zeros(16, np.float32)
        _check(lib().sf_get_setup(self._ctx, _fp(c), _fp(r)), "sf_get_setup", self._ctx)
        return c, r

    # rendering -------------------------------------------------------------
    def Render(self, **kw):
        """One deterministic frame into the device G-buffer (asynchronous)."""
        p = render_params(**kw)
        with self._mutex:
            _check(lib().sf_render(self._ctx, ctypes.byref(p)), "Render", self._ctx)

    def render_to(self, pos_ptr: int, nrm_ptr: int, min_t_ptr: int = 0, index_ptr: int = 0, **kw):
        """Render into caller-owned device buffers (e.g. torch tensor data_ptr())."""
        p = render_params(**kw)
        _check(lib().sf_render_to(self._ctx, ctypes.byref(p), ctypes.c_void_p(pos_ptr), ctypes.c_void_p(nrm_ptr),
                                  ctypes.c_void_p(min_t_ptr or None), ctypes.c_void_p(index_ptr or None)),
               "sf_render_to", self._ctx)

    def Synchronize(self):
        _check(lib().sf_synchronize(self._ctx), "sf_synchronize", self._ctx)

    def unpack_bands(self, stage_ptr: int, stage_rows: int, band_rows: int, band_count: int, first_member: int,
                     members: int, stream=None):
        """Packed band slabs on the device (render_to(..., packed=True, compact=True) of members first_member..)
        -> this context's G-buffer at frame positions (sf_unpack_bands), with the current view."""
        _check(lib().sf_unpack_bands(self._ctx, ctypes.c_void_p(stage_ptr), stage_rows, band_rows, band_count,
                                     first_member, members, stream), "sf_unpack_bands", self._ctx)

    def unpack_slabs(self, stage_ptr: int, bytes_per_pixel: int, stage_rows: int, band_rows: int, band_count: int,
                     first_member: int, members: int, stream=None):
        """Band slabs of either format (bytes_per_pixel 16: packed=1, 4: packed=2) -> this context's G-buffer
        (sf_unpack_slabs), with the current view."""
        _check(lib().sf_unpack_slabs(self._ctx, ctypes.c_void_p(stage_ptr), bytes_per_pixel, stage_rows, band_rows,
                                     band_count, first_member, members, stream), "sf_unpack_slabs", self._ctx)

    def slab_bytes(self) -> int:
        """Bytes per pixel of the smallest lossless band slab for the current view (sf_slab_bytes: 4 or 16)."""
        return int(lib().sf_slab_bytes(self._ctx))

    def device_buffers(self):
        ptrs = [ctypes.c_void_p() for _ in range(4)]
        _check(lib().sf_device_buffers(self._ctx, *[ctypes.byref(p) for p in ptrs]), "sf_device_buffers")
        return [p.value for p in ptrs]

    def download(self, aux: bool = False):
        """Synchronous D2H of the device G-buffer (+ minT and hit index channels if aux)."""
        H, W = self.height, self.width
        pos = np.empty((H, W, 4), np.float32)
        nrm = np.empty((H, W, 4), np.float32)
        mint = np.empty((H, W), np.float32) if aux else None
        idx = np.empty((H, W), np.uint32) if aux else None
        vp = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None
        self._raise_worker_error()
        with self._mutex:
            _check(lib().sf_download(self._ctx, vp(pos), vp(nrm), vp(mint), vp(idx)), "download", self._ctx)
        return pos, nrm, mint, idx

    def GetGBuffer(self) -> GBuffer:
        pos, nrm, _, _ = self.download()
        return GBuffer(pos, nrm)

    # reference variant ---------------------------------
    def SetVariant(self, variant):
        """'avx' / SF_VARIANT_AVX (default: LOD 70, 8-lane packets) or 'sse' / SF_VARIANT_SSE (LOD 60,
        4-lane packets, 2x2 frame-less footprint): the reference built without / with __ARCH_NO_AVX."""
        v = {"avx": SF_VARIANT_AVX, "sse": SF_VARIANT_SSE}.get(variant, variant)
        with self._mutex:
            _check(lib().sf_set_variant(self._ctx, int(v)), "SetVariant", self._ctx)

    def GetVariant(self) -> int:
        return lib().sf_get_variant(self._ctx)

    # transfer/interop ------------------------------------
    def pinned_gbuffer(self) -> GBuffer:
        """Host G-buffer arrays in the reference layout, page-locked for DMA (sf_host_register).
        Pass them to download_async; release with release_pinned()."""
        H, W = self.height, self.width
        g = GBuffer(np.zeros((H, W, 4), np.float32), np.zeros((H, W, 4), np.float32))
        for a in (g.positions, g.normals):
            _check(lib().sf_host_register(a.ctypes.data_as(ctypes.c_void_p), a.nbytes), "sf_host_register")
        self._pinned = getattr(self, "_pinned", []) + [g.positions, g.normals]
        return g

    def release_pinned(self):
        for a in getattr(self, "_pinned", []):
            lib().sf_host_unregister(a.ctypes.data_as(ctypes.c_void_p))
        self._pinned = []

    def download_async(self, g: GBuffer, stream: int | None = None):
        """Stream-ordered D2H of the G-buffer into `g` (pinned arrays from pinned_gbuffer());
        complete after Synchronize() (or the given stream's synchronisation)."""
        vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        with self._mutex:
            _check(lib().sf_download_async(self._ctx, vp(g.positions), vp(g.normals), None, None,
                                           ctypes.c_void_p(stream) if stream else None), "download_async", self._ctx)

    # SSAO post-process -----------------------------------
    def post_params(self, **kw) -> sf_post_params:
        """Reference defaults (SSAO.cpp:50-55, radius from the closest-hit stat, camera = view origin),
        overridden by keyword (sample_radius, intensity, scale, bias, normal_threshold, depth_threshold,
        camera_position, downscale, flags, stream)."""
        p = sf_post_params()
        _check(lib().sf_post_defaults(self._ctx, ctypes.byref(p)), "sf_post_defaults")
        for k, v in kw.items():
            if k == "camera_position":
                p.camera_position[:] = [float(x) for x in _f32(v, 3)]
            elif k == "stream":
                p.stream = v
            else:
                setattr(p, k, v)
        return p

    def PostProcess(self, pos_ptr: int = 0, nrm_ptr: int = 0, rgba_ptr: int = 0, ao_ptr: int = 0, **kw):
        """SSAO + blur x + blur y + final composite on the device (asynchronous). Pointers are device
        addresses (0 = the context's G-buffer / image buffer); ao_ptr receives the SSAO target."""
        p = self.post_params(**kw)
        vp = lambda x: ctypes.c_void_p(x) if x else None
        with self._mutex:
            _check(lib().sf_post_process(self._ctx, ctypes.byref(p), vp(pos_ptr), vp(nrm_ptr), vp(rgba_ptr),
                                         vp(ao_ptr)), "sf_post_process", self._ctx)

    def download_image(self) -> np.ndarray:
        """[H, W, 4] uint8 RGBA of the last PostProcess into the context image buffer."""
        img = np.empty((self.height, self.width, 4), np.uint8)
        with self._mutex:
            _check(lib().sf_download_image(self._ctx, img.ctypes.data_as(ctypes.c_void_p)), "sf_download_image",
                   self._ctx)
        return img

    @staticmethod
    def ssao_noise() -> np.ndarray:
        out = np.empty((64 * 64, 4), np.float32)
        _check(lib().sf_ssao_noise(_fp(out)), "sf_ssao_noise")
        return out

    def save_image(self, path: str, what: int = SF_DUMP_NORMALS) -> None:
        """Download this context's frame and write it as SF_DUMP_* (PPM of the post-processed image or
        of the normals, PFM of positions / normals) through the C ABI's sf_save_image."""
        with self._mutex:
            _check(lib().sf_save_image(self._ctx, os.fsencode(path), int(what)), "sf_save_image", self._ctx)

    @staticmethod
    def save_ppm(path: str, rgb) -> None:
        """Write an [H, W, 3] float image (0..1, clamped) as a binary PPM (8-bit), y = 0 on top."""
        a = np.clip(np.asarray(rgb, np.float32), 0.0, 1.0)
        b = (a * 255.0 + 0.5).astype(np.uint8)
        with open(path, "wb") as f:
            f.write(f"P6 {b.shape[1]} {b.shape[0]} 255\n".encode())
            f.write(np.ascontiguousarray(b[:, :, :3]).tobytes())

    def tile_trace(self, enable: bool | None = None):
        """Diagnostics: enable per-tile timing, or (enable=None) fetch [tiles, 3] uint64
        (start, end in 100 MHz ticks, (xcc << 32) | HW_ID) of the last render."""
        if enable is not None:
            _check(lib().sf_set_tile_trace(self._ctx, int(bool(enable))), "sf_set_tile_trace", self._ctx)
            return None
        n = ((self.width + 7) // 8) * ((self.height + 7) // 8)
        # tiles, SF_DIAG_SLOTS, units and waves (SF_FLAG_DIAG_UNITS): SF_TRACE_WORDS (sf_internal.h)
        out = np.zeros(15 * n + 16 + 2 * SF_DIAG_WAVES, np.uint64)
        _check(lib().sf_get_tile_trace(self._ctx, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), out.size),
               "sf_get_tile_trace", self._ctx)
        self.phase_sums = out[3 * n:3 * n + 16]   # segment cycle sums / event counts of diagnostic builds
        self.unit_trace = out[3 * n + 16:15 * n + 16].reshape(4 * n, 3)   # per order position (SF_FLAG_DIAG_UNITS)
        self.wave_trace = out[15 * n + 16:].reshape(SF_DIAG_WAVES, 2)   # per wave {start, end} (SF_FLAG_DIAG_UNITS)
        return out[:3 * n].reshape(n, 3)

    def tile_order(self):
        """Heavy-first schedule: (units, cost) uint32 arrays -- the work units (tile | part << 29) the
        next persistent render takes in order, and the last render's per-tile shader cycles they were
        computed from -- or None before any ordered render."""
        n = ((self.width + 7) // 8) * ((self.height + 7) // 8)
        order = np.zeros(4 * n, np.uint32)
        cost = np.zeros(n, np.uint32)
        P = ctypes.POINTER(ctypes.c_uint32)
        k = lib().sf_get_tile_order(self._ctx, order.ctypes.data_as(P), cost.ctypes.data_as(P), 4 * n)
        if k < 0:
            _check(k, "sf_get_tile_order", self._ctx)
        return (order[:k], cost) if k else None

    def kernel_timing(self, enable: bool | None = None, n: int = 64, period: int = 1):
        """Measurement: enable HIP events around the main trace kernel of every `period`-th render, or
        (enable=None) return the durations (ms) of the last n timed renders, oldest first."""
        if enable is not None:
            k = max(1, int(period)) if enable else 0
            _check(lib().sf_set_kernel_timing(self._ctx, k), "sf_set_kernel_timing", self._ctx)
            return None
        out = np.zeros(n, np.float32)
        k = lib().sf_kernel_times(self._ctx, out.ctypes.data_as(_F), n)
        if k < 0:
            _check(k, "sf_kernel_times", self._ctx)
        return out[:k]

    def kernel_clocks(self, n: int = 64):
        """Live shader clock (MHz) of the last n timed renders' trace kernels, oldest first (sf_kernel_clocks)."""
        out = np.zeros(n, np.float32)
        k = lib().sf_kernel_clocks(self._ctx, out.ctypes.data_as(_F), n)
        if k < 0:
            _check(k, "sf_kernel_clocks", self._ctx)
        return out[:k]

    # stats (Sphereflake.h:30-58) --------------------------------------------
    def stats(self) -> sf_stats:
        self._raise_worker_error()
        s = sf_stats()
        with self._mutex:
            _check(lib().sf_get_stats(self._ctx, ctypes.byref(s)), "sf_get_stats", self._ctx)
        return s

    def GetMaxDepthReached(self) -> int:
        return int(self.stats().max_depth)

    def ResetMaxDepthReached(self):
        _check(lib().sf_reset_max_depth(self._ctx), "ResetMaxDepthReached")

    def GetRaysPerSecond(self) -> int:
        """Rays traced since the last reset (the reference counter's meaning, main.cpp:285-291)."""
        return int(self.stats().rays)

    def ResetRaysPerSecond(self):
        _check(lib().sf_reset_rays(self._ctx), "ResetRaysPerSecond")

    def GetClosestSphereDistance(self) -> float:
        return float(self.stats().closest)

    def ResetClosestSphereDistance(self):
        _check(lib().sf_reset_closest(self._ctx), "ResetClosestSphereDistance")

    def reset_stats(self):
        """All three reference counters at once (ResetMaxDepthReached, ResetClosestSphereDistance,
        ResetRaysPerSecond)."""
        self.ResetMaxDepthReached()
        self.ResetClosestSphereDistance()
        self.ResetRaysPerSecond()

    # frame-less progressive mode (Sphereflake.cpp:67-74, 86-214) -------------
    def Progressive(self, seed: int, packets: int, counter0: int | None = None, stream=None):
        """Trace `packets` random 8-ray packets of one reference worker stream (seed, Sobol counter)."""
        c0 = self._counter if counter0 is None else int(counter0)
        with self._mutex:
            _check(lib().sf_progressive(self._ctx, seed & 0xffffffff, c0, packets, stream), "sf_progressive",
                   self._ctx)
        self._counter = c0 + packets

    def Initialize(self, seed: int | None = None, batch: int = 1 << 18):
        """Start the frame-less progressive loop on a host thread (reference Initialize(),
        Sphereflake.cpp:67-74; seeded from time() like Sphereflake.cpp:88-89 unless `seed` is given).
        The loop's first error stops it and is re-raised by the next GetGBuffer / stats call /
        Deinitialize."""
        import time
        if self._worker is not None:
            return
        self._raise_worker_error()
        self._seed = int(time.time()) if seed is None else int(seed)
        self._counter = 0
        self._stop.clear()

        def loop():
            try:
                while not self._stop.is_set():
                    with self._mutex:
                        _check(lib().sf_progressive(self._ctx, self._seed & 0xffffffff, self._counter, batch, None),
                               "sf_progressive", self._ctx)
                        _check(lib().sf_synchronize(self._ctx), "sf_synchronize", self._ctx)
                        self._counter += batch
            except Exception as e:   # kept for the caller's thread
                self._worker_error = e

        self._worker = threading.Thread(target=loop, daemon=True)
        self._worker.start()

    def Deinitialize(self):
        """Stop the frame-less loop and join it (the reference does this in its destructor)."""
        self._stop.set()
        if self._worker is not None:
            self._worker.join()
            self._worker = None
        self._raise_worker_error()

    def GetPacketsTraced(self) -> int:
        with self._mutex:
            return self._counter

    def _raise_worker_error(self):
        e, self._worker_error = getattr(self, "_worker_error", None), None
        if e is not None:
            raise RuntimeError(f"frame-less loop failed: {e}") from e


class SphereflakeGroup:
    """Single-process multi-GPU renderer (sf_group_*): interleaved 8-row bands traced on
    the member devices, gathered by strided peer copies into member 0's G-buffer. `devices` may repeat a
    device (n contexts on one GPU)."""

    def __init__(self, devices, width: int, height: int):
        self.width, self.height = int(width), int(height)
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        h = ctypes.c_void_p()
        _check(lib().sf_group_create(devs, len(devices), self.width, self.height, ctypes.byref(h)), "sf_group_create")
        self._g = h

    def close(self):
        if getattr(self, "_g", None):
            lib().sf_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, what):
        if rc != SF_OK:
            err = SphereflakeError(rc, what)
            if rc == SF_EHIP:
                err.hip_error = lib().sf_group_last_hip_error(self._g)
            raise err

    def size(self) -> int:
        return lib().sf_group_size(self._g)

    def member(self, k: int):
        """Member k's context handle (k = 0 holds the final G-buffer)."""
        return lib().sf_group_member(self._g, k)

    def SetView(self, origin, topLeft, topRight, bottomLeft):
        o, tl, tr, bl = (_vec3(v) for v in (origin, topLeft, topRight, bottomLeft))
        self._check(lib().sf_group_set_view(self._g, o, tl, tr, bl), "sf_group_set_view")

    def SetCamera(self, cam: Camera):
        self.SetView(*cam.corners())

    def SetVariant(self, variant):
        v = {"avx": SF_VARIANT_AVX, "sse": SF_VARIANT_SSE}.get(variant, variant)
        self._check(lib().sf_group_set_variant(self._g, int(v)), "sf_group_set_variant")

    def Render(self, band_rows: int = 8):
        self._check(lib().sf_group_render(self._g, int(band_rows)), "sf_group_render")

    def Synchronize(self):
        self._check(lib().sf_group_synchronize(self._g), "sf_group_synchronize")

    def download(self):
        H, W = self.height, self.width
        pos = np.empty((H, W, 4), np.float32)
        nrm = np.empty((H, W, 4), np.float32)
        self._check(lib().sf_group_download(self._g, pos.ctypes.data_as(ctypes.c_void_p),
                                            nrm.ctypes.data_as(ctypes.c_void_p)), "sf_group_download")
        return pos, nrm

    def member_kernel_timing(self, k: int, enable: bool | None = None, n: int = 64, period: int = 1):
        """Sphereflake.kernel_timing on member k's context (its main trace kernel)."""
        ctx = self.member(k)
        if enable is not None:
            _check(lib().sf_set_kernel_timing(ctx, max(1, int(period)) if enable else 0), "sf_set_kernel_timing", ctx)
            return None
        out = np.zeros(n, np.float32)
        got = lib().sf_kernel_times(ctx, out.ctypes.data_as(_F), n)
        if got < 0:
            _check(got, "sf_kernel_times", ctx)
        return out[:got]

    def reset_stats(self):
        self._check(lib().sf_group_reset_stats(self._g), "sf_group_reset_stats")

    def stats(self) -> sf_stats:
        """Over the members: max depth, closest distance, rays summed (accumulating across renders
        like the reference's counters until reset_stats)."""
        s = sf_stats()
        self._check(lib().sf_group_get_stats(self._g, ctypes.byref(s)), "sf_group_get_stats")
        return s

    def slab_bytes(self) -> int:
        """Bytes per pixel a member ships for the current view (4: hit index, 16: normal + minT)."""
        return int(lib().sf_group_slab_bytes(self._g))


def dist_unique_id() -> bytes:
    """A fresh RCCL unique id (sf_dist_unique_id): rank 0 makes one per slot and hands them to every rank."""
    buf = (ctypes.c_uint8 * SF_DIST_ID_BYTES)()
    _check(lib().sf_dist_unique_id(buf), "sf_dist_unique_id")
    return bytes(buf)


class SphereflakeDist:
    """One process per GPU (sf_dist_*): this rank's share of every frame (interleaved
    `band_rows`-row bands), gathered to rank 0 over RCCL as packed slabs; `slots` frames in flight. `ids`:
    slots x 128 bytes of dist_unique_id() from rank 0, or None: no communicator (nranks = 1, or this rank's bands
    of a distributed G-buffer via RenderBands only -- Render then raises SF_ESTATE)."""

    def __init__(self, device: int, width: int, height: int, rank: int = 0, nranks: int = 1, slots: int = 2,
                 ids: bytes | None = None, band_rows: int = 8):
        self.width, self.height, self.rank, self.nranks = int(width), int(height), int(rank), int(nranks)
        h = ctypes.c_void_p()
        idb = None
        if ids is not None:
            if len(ids) != slots * SF_DIST_ID_BYTES:
                raise ValueError("ids must hold slots x 128 bytes")
            idb = ctypes.create_string_buffer(bytes(ids), len(ids))
        _check(lib().sf_dist_create(int(device), self.width, self.height, int(band_rows), self.rank, self.nranks,
                                    int(slots), idb, ctypes.byref(h)), "sf_dist_create")
        self._d = h

    def close(self):
        if getattr(self, "_d", None):
            lib().sf_dist_destroy(self._d)
            self._d = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, what):
        if rc != SF_OK:
            err = SphereflakeError(rc, what)
            hip, nccl = ctypes.c_int(), ctypes.c_int()
            lib().sf_dist_last_error(self._d, ctypes.byref(hip), ctypes.byref(nccl))
            err.hip_error, err.rccl_error = hip.value, nccl.value
            raise err

    @property
    def slots(self) -> int:
        return lib().sf_dist_slots(self._d)

    def context(self, slot: int):
        return lib().sf_dist_context(self._d, int(slot))

    def last_slot(self) -> int:
        return lib().sf_dist_last_slot(self._d)

    def SetView(self, origin, topLeft, topRight, bottomLeft):
        o, tl, tr, bl = (_vec3(v) for v in (origin, topLeft, topRight, bottomLeft))
        self._check(lib().sf_dist_set_view(self._d, o, tl, tr, bl), "sf_dist_set_view")

    def SetCamera(self, cam: Camera):
        self.SetView(*cam.corners())

    def Render(self):
        """One frame: this rank's bands, gathered with the other ranks' into rank 0's G-buffer (RCCL)."""
        self._check(lib().sf_dist_render(self._d), "sf_dist_render")

    def RenderBands(self):
        """One frame as a distributed G-buffer: this rank's bands into its own slot G-buffer, no gather."""
        self._check(lib().sf_dist_render_bands(self._d), "sf_dist_render_bands")

    def RenderBandsFrames(self, views):
        """The next len(views) frames (each (origin, top-left, top-right, bottom-left)) as RenderBands would render
        them one by one, in ONE multi-frame persistent launch (sf_dist_render_bands_frames; len(views) <= slots)."""
        v = _views12(views)
        self._check(lib().sf_dist_render_bands_frames(self._d, len(views), _fp(v)), "sf_dist_render_bands_frames")

    def download_slot(self, slot: int):
        """The G-buffer of one slot's context on this rank (synchronises)."""
        H, W = self.height, self.width
        pos = np.empty((H, W, 4), np.float32)
        nrm = np.empty((H, W, 4), np.float32)
        ctx = self.context(slot)
        _check(lib().sf_download(ctx, pos.ctypes.data_as(ctypes.c_void_p), nrm.ctypes.data_as(ctypes.c_void_p),
                                 None, None), "sf_download", ctx)
        return pos, nrm

    def Synchronize(self):
        self._check(lib().sf_dist_synchronize(self._d), "sf_dist_synchronize")

    def download(self):
        """Rank 0: the last frame's G-buffer (synchronises)."""
        H, W = self.height, self.width
        pos = np.empty((H, W, 4), np.float32)
        nrm = np.empty((H, W, 4), np.float32)
        self._check(lib().sf_dist_download(self._d, pos.ctypes.data_as(ctypes.c_void_p),
                                           nrm.ctypes.data_as(ctypes.c_void_p)), "sf_dist_download")
        return pos, nrm

    def stats(self) -> sf_stats:
        """Over this rank's slots, and over the ranks when made with ids (then collective: every rank calls it);
        without ids the caller combines the ranks' stats."""
        s = sf_stats()
        self._check(lib().sf_dist_get_stats(self._d, ctypes.byref(s)), "sf_dist_get_stats")
        return s

    def reset_stats(self):
        self._check(lib().sf_dist_reset_stats(self._d), "sf_dist_reset_stats")

    def kernel_timing(self, slot: int, enable: bool | None = None, n: int = 64, period: int = 1):
        """Trace-kernel events of one slot's context (Sphereflake.kernel_timing)."""
        ctx = self.context(slot)
        if enable is not None:
            _check(lib().sf_set_kernel_timing(ctx, max(1, int(period)) if enable else 0), "sf_set_kernel_timing", ctx)
            return None
        out = np.zeros(n, np.float32)
        got = lib().sf_kernel_times(ctx, out.ctypes.data_as(_F), n)
        if got < 0:
            _check(got, "sf_kernel_times", ctx)
        return out[:got]

    def comm_info(self, slot: int = 0):
        """(ncclCommCount, ncclCommUserRank, ncclCommCuDevice) of a slot's RCCL communicator (sf_dist_comm_info)."""
        v = [ctypes.c_int() for _ in range(3)]
        self._check(lib().sf_dist_comm_info(self._d, int(slot), *[ctypes.byref(x) for x in v]), "sf_dist_comm_info")
        return tuple(x.value for x in v)

    def slab_bytes(self) -> int:
        """Bytes per pixel the gather ships for the current view (4: hit index, 16: normal + minT)."""
        return int(lib().sf_dist_slab_bytes(self._d))

    def kernel_clocks(self, slot: int, n: int = 64):
        ctx = self.context(slot)
        out = np.zeros(n, np.float32)
        got = lib().sf_kernel_clocks(ctx, out.ctypes.data_as(_F), n)
        if got < 0:
            _check(got, "sf_kernel_clocks", ctx)
        return out[:got]
