"""MI355X-native Monte Carlo path tracer -- host-side mirror of the reference's render interface.

The reference (luotong96/Monte_Carlo_Path_Tracing) renders in `main()` (main.cpp:497-600):
load `Myobj veach` / `Mylight lights` (main.cpp:23-24, 500-504), set the camera (main.cpp:507-510),
trace one pixel-centre ray per pixel and average `spp` calls of `shade_with_mis` /
`shade_with_brdf` (main.cpp:557-588), tone-map (main.cpp:583) and save `test.bmp` (main.cpp:596).

Here the same steps are `Scene.load`, `Camera.reference`, `render(scene, camera, spp, mode)`,
`tone_map` and `write_bmp`, all backed by the C ABI of `libmcpt_hip.so` (include/mcpt.h), whose
hot path is hand-written HIP for gfx950.  There is no CPU fallback: every call fails loudly when
the native library (or, for rendering, a GPU) is missing.
"""
import ctypes as C
import os

import numpy as np

__all__ = ["Scene", "Camera", "Comm", "render", "render_device", "closest_hit", "light_prep", "primary_hits",
           "tone_map", "write_bmp", "MODE_MIS", "MODE_BRDF", "MODE_SHADE", "MODE_SHADE_AREA", "ACCEL_BVH", "ACCEL_GRID", "Stats", "MCPTError", "LIB_PATH", "lib"]

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCPT_LIB_PATH") or os.path.join(HERE, "libmcpt_hip.so")  # override: A/B of two builds
MODE_MIS, MODE_BRDF, MODE_SHADE = 0, 1, 2  # shade_with_mis / shade_with_brdf / shade (main.cpp:402/348/269)
MODE_SHADE_AREA = 3  # shade with select_a_point_from_lights (Mylight.cpp:102-160; main.cpp:296)
MODES = {"mis": MODE_MIS, "brdf": MODE_BRDF, "shade": MODE_SHADE, "shade_area": MODE_SHADE_AREA}
ACCEL_BVH, ACCEL_GRID = 0, 1  # mcpt_render_opts.accel: BVH, or the reference's uniform grid (Myobj.cpp:78-162)
HIT_LIGHT_ONLY, HIT_GRID = 1, 2  # mcpt_closest_hit flags
DEFAULT_SEED = 20240430
MCPT_VERSION = 20200  # include/mcpt.h MCPT_VERSION this mirror is written against
COMM_ID_BYTES = 128  # MCPT_COMM_ID_BYTES
STATS_MAX_DEVICES = 16  # MCPT_STATS_MAX_DEVICES


class MCPTError(RuntimeError):
    pass


class Camera(C.Structure):
    """mcpt_camera: main.cpp:507-510,547-564 generalised to width x height."""
    _fields_ = [("eye", C.c_double * 3), ("lookat", C.c_double * 3), ("up", C.c_double * 3),
                ("fovy", C.c_double), ("dist_scale", C.c_double), ("width", C.c_int32), ("height", C.c_int32)]

    @classmethod
    def reference(cls, width=1280, height=720, dist_scale=2.0):
        """The hard-coded Veach camera of main.cpp:507-510 (eye pulled back 2x)."""
        c = cls()
        c.eye[:] = (28.2792, 5.2, 1.23612e-06)
        c.lookat[:] = (0.0, 2.8, 0.0)
        c.up[:] = (0.0, 1.0, 0.0)
        c.fovy = 20.1143
        c.dist_scale = dist_scale
        c.width, c.height = int(width), int(height)
        return c


class RenderOpts(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("spp", C.c_int32), ("sample_begin", C.c_int32),
                ("sample_end", C.c_int32), ("mode", C.c_int32),
                ("seed", C.c_uint64), ("samples_per_launch", C.c_int32), ("queue_factor", C.c_int32),
                ("device", C.c_int32), ("accel", C.c_int32), ("progress", C.c_void_p),
                ("progress_user", C.c_void_p), ("flags", C.c_int32), ("num_devices", C.c_int32),
                ("devices", C.POINTER(C.c_int32)), ("comm", C.c_void_p), ("stats_size", C.c_uint32)]
RENDER_NO_BACKFACE_STATS = 1  # mcpt_render_opts.flags (include/mcpt.h)
RENDER_FRESH_PDF = 2  # shade_with_mis: the node's own light pdf instead of the reference's stale one
RENDER_PRECISION_FP32 = 4  # opt-in FP32_STABLE light prep (packed-fp32 weights, fp64 sums); default FP64_LIGHT
DEBUG_SPLIT_BRDF, DEBUG_NO_ROOT_CACHE, DEBUG_COUNT_TRAVERSAL = 1 << 16, 1 << 17, 1 << 18  # include/mcpt_debug.h
DEBUG_SHARD_RANKS = 1 << 19  # device lists: every entry its own communicator rank (tests/collshim)
DEBUG_RAYS_PERSIST = 1 << 20  # MIS / shade ray sets through the persistent refilling traversal on every scene
DEBUG_RAYS_CW8 = 1 << 21  # the persistent traversal walks the 8-wide compressed trees (k_rays_cw8)
DEBUG_FUSED_CULL = 1 << 22  # MIS children's prep: cheap stages inside k_prep_pk2 (variant 8) instead of k_prep_cull_lanes
DEBUG_NO_EXACT_DEFER = 1 << 23  # k_prep_exact recomputes same-launch duplicate roots instead of deferring them
DEBUG_HIT_CW8 = 1 << 8  # mcpt_closest_hit: trace through the 8-wide trees


PROGRESS_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, C.c_uint64)


class Stats(C.Structure):
    _fields_ = [("seconds", C.c_double), ("camera_samples", C.c_uint64), ("shading_nodes", C.c_uint64),
                ("light_evals_survived", C.c_uint64), ("rays", C.c_uint64), ("light_rays", C.c_uint64),
                ("generations", C.c_uint64), ("prep_seconds", C.c_double), ("prep_launches", C.c_uint64),
                ("light_evals_total", C.c_uint64), ("light_evals_culled_backface", C.c_uint64),
                ("light_evals_culled_plane", C.c_uint64), ("light_evals_candidates", C.c_uint64),
                ("prep_full_nodes", C.c_uint64), ("prep_cached_nodes", C.c_uint64), ("prep_cache_points", C.c_uint64),
                ("spilled_nodes", C.c_uint64), ("reduce_seconds", C.c_double), ("devices_used", C.c_int32),
                ("trace_seconds", C.c_double), ("trace_launches", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("prep_exact_nodes", C.c_uint64), ("cache_build_seconds", C.c_double),
                ("prep_band_nodes", C.c_uint64), ("comm_init_seconds", C.c_double),
                ("device_setup_seconds", C.c_double), ("device_seconds", C.c_double * STATS_MAX_DEVICES)]

    def as_dict(self):
        """scalar fields (summable); device_seconds is in per_device_seconds()"""
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "device_seconds"}

    def per_device_seconds(self):
        """device_seconds[:devices_used]: each rank's shard wall time (setup and reduce excluded)"""
        return [float(v) for v in self.device_seconds[:max(1, min(self.devices_used, STATS_MAX_DEVICES))]]


_lib = None

# every symbol include/mcpt.h declares (tests check the .so exports them all)
EXPORTS = ["mcpt_version", "mcpt_last_error", "mcpt_scene_load", "mcpt_scene_create", "mcpt_scene_destroy",
           "mcpt_scene_counts", "mcpt_scene_accel_bytes", "mcpt_scene_arrays", "mcpt_scene_camera", "mcpt_scene_meshing", "mcpt_scene_grid_info",
           "mcpt_render_opts_init", "mcpt_render", "mcpt_render_device",
           "mcpt_closest_hit", "mcpt_light_prep", "mcpt_primary_hits", "mcpt_tone_map",
           "mcpt_write_bmp", "mcpt_comm_unique_id", "mcpt_comm_init_rank", "mcpt_comm_destroy"]
DEBUG_EXPORTS = ["mcpt_debug_prep_bench", "mcpt_debug_tri_filter", "mcpt_debug_light_prep_exact", "mcpt_debug_light_literal",
                 "mcpt_debug_set_collective_lib", "mcpt_debug_bvh8_check", "mcpt_debug_bvh4_check"]  # include/mcpt_debug.h


def lib():
    """The native library; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MCPTError("libmcpt_hip.so not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                            "or `make -C monte_carlo_path_tracing_amd/csrc`")
        # One HIP runtime per process: torch wheels bundle their own libamdhip64.so.7 /
        # libhsa-runtime64.so.1 (same sonames as /opt/rocm's).  Loading torch first makes this
        # library bind to torch's runtime, so device pointers and streams are shared; loading
        # /opt/rocm's runtime first would leave torch without a usable GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        P, I, D = C.c_void_p, C.c_int32, C.c_double
        dp = np.ctypeslib.ndpointer(np.float64, flags="C")
        fp = np.ctypeslib.ndpointer(np.float32, flags="C")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C")
        u8 = np.ctypeslib.ndpointer(np.uint8, flags="C")
        L.mcpt_version.restype = C.c_int
        L.mcpt_last_error.restype = C.c_char_p
        L.mcpt_scene_load.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(P)]
        L.mcpt_scene_create.argtypes = [P, C.POINTER(P)]
        L.mcpt_scene_destroy.argtypes = [P]
        L.mcpt_scene_destroy.restype = None
        L.mcpt_scene_counts.argtypes = [P, C.POINTER(I), C.POINTER(I), C.POINTER(I)]
        L.mcpt_scene_accel_bytes.argtypes = [P, C.POINTER(C.c_uint64)]
        L.mcpt_scene_arrays.argtypes = [P, fp, fp, ip, fp, ip, dp, dp]
        L.mcpt_scene_camera.argtypes = [P, C.POINTER(Camera)]
        L.mcpt_scene_meshing.argtypes = [P, dp, I]
        L.mcpt_scene_grid_info.argtypes = [P, dp, ip]
        L.mcpt_render_opts_init.argtypes = [C.POINTER(RenderOpts)]
        L.mcpt_render_opts_init.restype = None
        L.mcpt_render.argtypes = [P, C.POINTER(Camera), C.POINTER(RenderOpts), dp, C.POINTER(Stats)]
        L.mcpt_render_device.argtypes = [P, C.POINTER(Camera), C.POINTER(RenderOpts), C.c_void_p, C.POINTER(Stats)]
        L.mcpt_closest_hit.argtypes = [P, I, dp, dp, ip, I, ip, dp]
        L.mcpt_light_prep.argtypes = [P, I, dp, dp, dp, dp, ip, ip]
        L.mcpt_primary_hits.argtypes = [P, C.POINTER(Camera), ip, dp]
        # debug entry points (include/mcpt_debug.h): bound when present, so an older build can still
        # be timed against this one through MCPT_LIB_PATH (tools/ab_run.sh)
        dbg = {"mcpt_debug_prep_bench": [P, I, dp, dp, dp, I, I, C.POINTER(C.c_double), dp, ip],
               "mcpt_debug_tri_filter": [I, fp, dp, dp, fp, ip, fp],
               "mcpt_debug_light_prep_exact": [P, I, dp, dp, dp, dp, ip, ip],
               "mcpt_debug_light_literal": [P, dp, dp, dp],
               "mcpt_debug_set_collective_lib": [C.c_char_p],
               "mcpt_debug_bvh8_check": [P, I, np.ctypeslib.ndpointer(np.int64, flags="C")],
               "mcpt_debug_bvh4_check": [P, I, np.ctypeslib.ndpointer(np.int64, flags="C")]}
        for name, argt in dbg.items():
            if hasattr(L, name):
                getattr(L, name).argtypes = argt
        L.mcpt_tone_map.argtypes = [dp, I, I, D, D, u8]
        L.mcpt_write_bmp.argtypes = [C.c_char_p, u8, I, I]
        L.mcpt_comm_unique_id.argtypes = [C.c_char_p]
        L.mcpt_comm_init_rank.argtypes = [I, I, C.c_char_p, I, C.POINTER(P)]
        L.mcpt_comm_destroy.argtypes = [P]
        L.mcpt_comm_destroy.restype = None
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise MCPTError("mcpt error %d: %s" % (rc, lib().mcpt_last_error().decode()))


def _d(x, shape=None):
    a = np.ascontiguousarray(x, dtype=np.float64)
    return a if shape is None else a.reshape(shape)


class Scene:
    """Myobj + Mylight: an OBJ/MTL scene and its <light mtlname radiance> XML (main.cpp:500-504)."""

    def __init__(self, handle):
        self.h = handle
        # bound now: at interpreter shutdown the module's globals (lib) may already be gone when __del__ runs
        self._destroy = lib().mcpt_scene_destroy
        f, m, n = C.c_int32(), C.c_int32(), C.c_int32()
        _check(lib().mcpt_scene_counts(self.h, C.byref(f), C.byref(m), C.byref(n)))
        self.nfacets, self.nmaterials, self.nlights = f.value, m.value, n.value

    @classmethod
    def load(cls, obj_path, xml_path):
        h = C.c_void_p()
        _check(lib().mcpt_scene_load(os.fsencode(obj_path), os.fsencode(xml_path), C.byref(h)))
        return cls(h)

    def close(self):
        if getattr(self, "h", None):
            self._destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def arrays(self):
        F, M, NL = self.nfacets, self.nmaterials, self.nlights
        pos, nrm = np.zeros((F, 9), np.float32), np.zeros((F, 9), np.float32)
        mat, mtl = np.zeros(F, np.int32), np.zeros((M, 7), np.float32)
        lf, lr, un = np.zeros(max(NL, 1), np.int32), np.zeros((max(NL, 1), 3)), np.zeros((F, 3))
        _check(lib().mcpt_scene_arrays(self.h, pos, nrm, mat, mtl, lf, lr, un))
        return dict(positions=pos, normals=nrm, material_id=mat, materials=mtl, light_facet=lf[:NL],
                    light_radiance=lr[:NL], unique_normal=un)

    def meshing(self, eye, n0=100000):
        """Myobj::cal_scene_boundingbox(eye) + Myobj::meshing(n0) (Myobj.cpp:78-162): the reference's
        uniform grid, for closest_hit(..., grid=True)."""
        _check(lib().mcpt_scene_meshing(self.h, _d(eye, (3,)), int(n0)))

    def grid_info(self):
        """((xmin, xmax, ymin, ymax, zmin, zmax, cell edge), cells per axis) of the current grid"""
        box, cells = np.zeros(7), np.zeros(3, np.int32)
        _check(lib().mcpt_scene_grid_info(self.h, box, cells))
        return box, cells

    def accel_bytes(self):
        """device bytes of the BVHs the traversal reads (mcpt_scene_accel_bytes)"""
        b = C.c_uint64()
        _check(lib().mcpt_scene_accel_bytes(self.h, C.byref(b)))
        return b.value

    def camera(self):
        c = Camera()
        _check(lib().mcpt_scene_camera(self.h, C.byref(c)))
        return c


class Comm:
    """mcpt_comm: this process's rank of a multi-process RCCL communicator owned by the library
    (one process per GPU).  Rank 0 calls Comm.unique_id(); the caller broadcasts the bytes (e.g.
    torch.distributed.broadcast_object_list); every rank then constructs Comm(nranks, rank, id, device).
    Renders with comm=... render this rank's share of the job's sample range and end with ONE
    ncclReduce(sum) into rank 0's buffer."""

    def __init__(self, nranks, rank, uid, device=-1):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("comm id must be %d bytes" % COMM_ID_BYTES)
        h = C.c_void_p()
        self._destroy = lib().mcpt_comm_destroy
        _check(lib().mcpt_comm_init_rank(int(nranks), int(rank), bytes(uid), int(device), C.byref(h)))
        self.h, self.nranks, self.rank = h, int(nranks), int(rank)

    @staticmethod
    def unique_id():
        buf = C.create_string_buffer(COMM_ID_BYTES)
        _check(lib().mcpt_comm_unique_id(buf))
        return buf.raw

    def close(self):
        if getattr(self, "h", None):
            self._destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def set_collective_lib(path):
    """Test infrastructure (include/mcpt_debug.h): use the NCCL-API library at `path` (the host-memory
    collective tests/collshim/libmcpt_collshim.so) instead of RCCL for this process's communicators, so
    several ranks can share one GPU.  Must precede the first Comm / device-list render."""
    _check(lib().mcpt_debug_set_collective_lib(os.fsencode(path)))


def _opts(spp, mode, seed, sample_range, device, samples_per_launch, queue_factor, progress=None, accel="bvh",
          flags=0, devices=None, comm=None):
    """progress(done, total) -> truthy to cancel; the ctypes thunk is kept on the returned struct.
    devices: list of device ordinals (one process, several GPUs); comm: a Comm (one process per GPU)."""
    o = RenderOpts()
    lib().mcpt_render_opts_init(C.byref(o))
    o.flags = int(flags)
    if devices is not None:
        o._devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        o.num_devices = len(devices)
        o.devices = C.cast(o._devs, C.POINTER(C.c_int32))
    if comm is not None:
        o.comm = comm.h
    a = {"bvh": ACCEL_BVH, "grid": ACCEL_GRID}.get(accel, -1) if isinstance(accel, str) else int(accel)
    if a not in (ACCEL_BVH, ACCEL_GRID):
        raise ValueError("accel must be 'bvh' or 'grid'")
    o.accel = a
    if progress is not None:
        o._thunk = PROGRESS_FN(lambda _u, done, total: 1 if progress(int(done), int(total)) else 0)
        o.progress = C.cast(o._thunk, C.c_void_p)
    o.spp = int(spp)
    o.sample_begin = o.sample_end = 0
    m = MODES.get(mode, -1) if isinstance(mode, str) else int(mode)
    if m not in MODES.values():
        raise ValueError("mode must be one of %s" % sorted(MODES))
    o.mode = m
    o.seed = int(seed)
    if sample_range is not None:
        o.sample_begin, o.sample_end = int(sample_range[0]), int(sample_range[1])
    o.device = -1 if device is None else int(device)
    o.samples_per_launch = int(samples_per_launch or 0)
    o.queue_factor = int(queue_factor or 0)
    return o


def render(scene, camera, spp, mode="mis", seed=DEFAULT_SEED, sample_range=None, out=None, device=None,
           samples_per_launch=0, queue_factor=0, progress=None, accel="bvh", devices=None, comm=None, flags=0):
    """render(scene, camera, spp, mode) -- main.cpp:547-588.  Returns (H x W x 3 fp64 radiance, Stats).

    Adds sum_k L_k / spp over samples k in `sample_range` (default all) into `out` (zeros if None).
    progress(samples_dispatched, samples_total), called after every wavefront generation, replaces
    the reference's per-row progress output; a truthy return cancels (MCPTError, partial sum).
    accel="grid" traces every ray through the reference's uniform grid (Myobj.cpp:78-162) instead of
    the BVH: hit-for-hit the reference's traversal, crack included.
    devices=[d0, d1, ...] shards the sample range over several GPUs of this process (one thread and
    stream each; a device may repeat) and sums them with one RCCL reduce; comm=Comm(...) renders this
    rank's share and reduces to rank 0 (see mcpt_render_opts in include/mcpt.h)."""
    if out is None:
        out = np.zeros((camera.height, camera.width, 3))
    assert out.dtype == np.float64 and out.flags.c_contiguous and out.shape == (camera.height, camera.width, 3)
    st = Stats()
    o = _opts(spp, mode, seed, sample_range, device, samples_per_launch, queue_factor, progress, accel, flags,
              devices, comm)
    _check(lib().mcpt_render(scene.h, C.byref(camera), C.byref(o), out.reshape(-1), C.byref(st)))
    return out, st


def render_device(scene, camera, spp, dev_ptr, mode="mis", seed=DEFAULT_SEED, sample_range=None, device=None,
                  samples_per_launch=0, queue_factor=0, progress=None, accel="bvh", flags=0, devices=None, comm=None):
    """Accumulate into a device buffer of H*W*3 doubles (e.g. a torch.float64 CUDA tensor's data_ptr()).
    flags: RENDER_NO_BACKFACE_STATS skips the light-side cull statistic (mcpt_render_opts.flags)."""
    st = Stats()
    o = _opts(spp, mode, seed, sample_range, device, samples_per_launch, queue_factor, progress, accel, flags,
              devices, comm)
    _check(lib().mcpt_render_device(scene.h, C.byref(camera), C.byref(o), C.c_void_p(int(dev_ptr)), C.byref(st)))
    return st


def closest_hit(scene, ro, rd, exclude=None, light_only=False, grid=False, wide=False):
    """Myobj::closet_ray_intersect (Myobj.cpp:334) / ..._light_triangle (:476) for a batch of rays.
    grid=True traverses the reference's uniform grid of Scene.meshing (crack included), else the BVH;
    wide=True (diagnostics) the 8-wide compressed BVH of the persistent traversal (k_rays_cw8)."""
    ro, rd = _d(ro, (-1, 3)), _d(rd, (-1, 3))
    n = ro.shape[0]
    ex = np.full(n, -1, np.int32) if exclude is None else np.ascontiguousarray(exclude, np.int32)
    f, tbg = np.zeros(n, np.int32), np.zeros((n, 3))
    flags = (HIT_LIGHT_ONLY if light_only else 0) | (HIT_GRID if grid else 0) | (DEBUG_HIT_CW8 if wide else 0)
    _check(lib().mcpt_closest_hit(scene.h, n, ro, rd, ex, flags, f, tbg))
    return f, tbg


def light_prep(scene, x1, normal, u):
    """Mylight::prepared_for_lights_spherical_triangle_sampling at n points + the inverse-CDF pick."""
    x1, normal, u = _d(x1, (-1, 3)), _d(normal, (-1, 3)), _d(u, (-1,))
    n = x1.shape[0]
    ws, cnt, pick = np.zeros(n), np.zeros(n, np.int32), np.zeros(n, np.int32)
    _check(lib().mcpt_light_prep(scene.h, n, x1, normal, u, ws, cnt, pick))
    return ws, cnt, pick


def debug_light_prep_exact(scene, x1, normal, u):
    """Diagnostics: light_prep with every point through the exact fallback alone (the reference's
    literal cull chain and weights, summed in index order; include/mcpt_debug.h)."""
    x1, normal, u = _d(x1, (-1, 3)), _d(normal, (-1, 3)), _d(u, (-1,))
    n = x1.shape[0]
    ws, cnt, pick = np.zeros(n), np.zeros(n, np.int32), np.zeros(n, np.int32)
    _check(lib().mcpt_debug_light_prep_exact(scene.h, n, x1, normal, u, ws, cnt, pick))
    return ws, cnt, pick


def debug_light_literal(scene, x1, normal):
    """Diagnostics: the literal cull chain's intermediates for every light at one point (N_L x 20)."""
    out = np.zeros((scene.nlights, 20))
    _check(lib().mcpt_debug_light_literal(scene.h, _d(x1, (3,)), _d(normal, (3,)), out.reshape(-1)))
    return out


def debug_bvh8_check(scene, light_only=False):
    """Diagnostics (host only): the 8-wide tree against its binary tree (include/mcpt_debug.h).  Returns dict
    nodes, tris, facets, duplicates, errors, depth."""
    out = np.zeros(6, np.int64)
    _check(lib().mcpt_debug_bvh8_check(scene.h, 1 if light_only else 0, out))
    return dict(zip(("nodes", "tris", "facets", "duplicates", "errors", "depth"), (int(v) for v in out)))


def debug_bvh4_check(scene, light_only=False):
    """Diagnostics (host only): the 4-wide tree every traversal reads and its quantized form against the
    binary tree (include/mcpt_debug.h).  Returns dict nodes, tris, facets, duplicates, errors, depth."""
    out = np.zeros(6, np.int64)
    _check(lib().mcpt_debug_bvh4_check(scene.h, 1 if light_only else 0, out))
    return dict(zip(("nodes", "tris", "facets", "duplicates", "errors", "depth"), (int(v) for v in out)))


def debug_tri_filter(tri, ro, rd, tlim=None):
    """Diagnostics (host only): the traversal's fp32 triangle pre-test on (triangle, ray) pairs.
    Returns (verdict, tup): 0 = the fp64 test surely rejects (or the hit is surely beyond tlim),
    2 = it surely accepts with t <= tup, 1 = undecided (include/mcpt_debug.h)."""
    tri = np.ascontiguousarray(tri, np.float32).reshape(-1, 9)
    n = tri.shape[0]
    ro, rd = _d(ro, (-1, 3)), _d(rd, (-1, 3))
    tl = np.full(n, np.finfo(np.float32).max, np.float32) if tlim is None else np.ascontiguousarray(tlim, np.float32)
    verdict, tup = np.zeros(n, np.int32), np.zeros(n, np.float32)
    _check(lib().mcpt_debug_tri_filter(n, tri, ro, rd, tl, verdict, tup))
    return verdict, tup


def debug_prep_bench(scene, x1, normal, u, variant=-1, iters=5):
    """Diagnostics: mean ms per launch of a light-prep kernel variant (see include/mcpt.h)."""
    x1, normal, u = _d(x1, (-1, 3)), _d(normal, (-1, 3)), _d(u, (-1,))
    n = x1.shape[0]
    ms, ws, pick = C.c_double(), np.zeros(n), np.zeros(n, np.int32)
    _check(lib().mcpt_debug_prep_bench(scene.h, n, x1, normal, u, int(variant), int(iters), C.byref(ms), ws, pick))
    return ms.value, ws, pick


def primary_hits(scene, camera):
    n = camera.width * camera.height
    f, tbg = np.zeros(n, np.int32), np.zeros((n, 3))
    _check(lib().mcpt_primary_hits(scene.h, C.byref(camera), f, tbg))
    return f, tbg


def tone_map(hdr, max_radiance=380.0, gamma=0.25):
    """RadianceRGB::tone_mapping(380, 0.25) of main.cpp:583 over a whole H x W x 3 frame."""
    hdr = np.ascontiguousarray(hdr, np.float64)
    H, W = hdr.shape[:2]
    out = np.zeros((H, W, 3), np.uint8)
    _check(lib().mcpt_tone_map(hdr.reshape(-1), W, H, max_radiance, gamma, out.reshape(-1)))
    return out


def write_bmp(path, rgb8):
    """The 32-bpp bottom-up BMP layout of the reference's test.bmp (main.cpp:596)."""
    rgb8 = np.ascontiguousarray(rgb8, np.uint8)
    H, W = rgb8.shape[:2]
    _check(lib().mcpt_write_bmp(os.fsencode(path), rgb8.reshape(-1), W, H))
