"""TEST INFRASTRUCTURE ONLY -- ctypes view of oracle/liboracle.so (the C restatement).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCPT_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")  # override: the sanitizer build

MODE_MIS, MODE_BRDF, MODE_SHADE, MODE_SHADE_AREA = 0, 1, 2, 3  # ORC_MODE_* (mcpt_oracle.h)
FLAG_FRESH_PDF = 0x200  # ORC_FLAG_FRESH_PDF: or into MODE_MIS for the node's own light pdf instead of the reference's stale one
RNG_REF, RNG_COUNTER = 0, 1


class Camera(C.Structure):
    _fields_ = [("eye", C.c_double * 3), ("lookat", C.c_double * 3), ("up", C.c_double * 3),
                ("fovy", C.c_double), ("dist_scale", C.c_double), ("width", C.c_int), ("height", C.c_int)]


def reference_camera(width, height, dist_scale=2.0):
    """main.cpp:507-510 (Veach eye/lookat, eye pulled back 2x), README.md:339-343."""
    c = Camera()
    c.eye[:] = (28.2792, 5.2, 1.23612e-06)
    c.lookat[:] = (0.0, 2.8, 0.0)
    c.up[:] = (0.0, 1.0, 0.0)
    c.fovy = 20.1143
    c.dist_scale = dist_scale
    c.width, c.height = width, height
    return c


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        dp = np.ctypeslib.ndpointer(np.float64, flags="C")
        fp = np.ctypeslib.ndpointer(np.float32, flags="C")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C")
        up = np.ctypeslib.ndpointer(np.uint64, flags="C")
        L.orc_scene_load.restype = P
        L.orc_scene_load.argtypes = [C.c_char_p, C.c_char_p]
        L.orc_scene_free.argtypes = [P]
        L.orc_last_error.restype = C.c_char_p
        L.orc_scene_counts.argtypes = [P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_scene_facets.argtypes = [P, fp, ip, ip, dp]
        L.orc_scene_materials.argtypes = [P, fp]
        L.orc_scene_lights.argtypes = [P, ip, dp]
        L.orc_scene_camera.argtypes = [P, C.POINTER(Camera)]
        L.orc_grid_build.argtypes = [P, dp, C.c_int]
        L.orc_grid_info.argtypes = [P, dp]
        for fn in (L.orc_closest_hit, L.orc_closest_light_hit, L.orc_intersect_triangle):
            fn.restype = C.c_int
            fn.argtypes = [P, dp, dp, C.c_int, dp]
        L.orc_brdf_phong.argtypes = [dp, dp, dp, dp, dp, C.c_double, dp]
        L.orc_phong_pdf.restype = C.c_double
        L.orc_phong_pdf.argtypes = [dp, dp, dp, dp, dp, C.c_double]
        L.orc_sample_phong_ref.argtypes = [C.c_uint64, dp, dp, dp, dp, C.c_double, dp]
        L.orc_sample_phong_u.argtypes = [dp, dp, dp, dp, C.c_double, C.c_double, C.c_double, C.c_double, dp]
        L.orc_light_prep.restype = C.c_double
        L.orc_light_prep.argtypes = [P, dp, dp, C.POINTER(C.c_int), ip, dp]
        L.orc_light_sample_ref.argtypes = [P, C.c_uint64, dp, dp, dp]
        L.orc_light_sample_u.argtypes = [P, dp, dp, C.c_double, C.c_double, C.c_double, dp]
        L.orc_light_pdf.restype = C.c_double
        L.orc_light_pdf.argtypes = [P, dp, dp, C.c_int]
        L.orc_tone_map.argtypes = [dp, C.c_double, C.c_double, ip]
        L.orc_camera_ray.argtypes = [C.POINTER(Camera), C.c_int, C.c_int, dp, dp]
        L.orc_shade_sample.argtypes = [P, C.POINTER(Camera), C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int,
                                       C.c_int, dp, C.POINTER(C.c_uint64)]
        L.orc_render.restype = C.c_int
        L.orc_render.argtypes = [P, C.POINTER(Camera), C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.c_int, dp, up]
        L.orc_depth_study.restype = C.c_int
        L.orc_depth_study.argtypes = [P, C.POINTER(Camera), C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      dp, up]
        L.orc_counter_uniform.restype = C.c_double
        L.orc_counter_uniform.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32]
        _lib = L
    return _lib


def _v(x):
    return np.ascontiguousarray(x, dtype=np.float64)


class Scene:
    """Oracle scene: loads OBJ/MTL/XML like Myobj::read + Mylight::read/gather_light_triangles."""

    def __init__(self, obj_path, xml_path):
        L = lib()
        self.h = L.orc_scene_load(obj_path.encode(), xml_path.encode())
        if not self.h:
            raise RuntimeError("oracle scene load failed: %s" % L.orc_last_error().decode())
        f, m, n = C.c_int(), C.c_int(), C.c_int()
        L.orc_scene_counts(self.h, C.byref(f), C.byref(m), C.byref(n))
        self.nfacets, self.nmaterials, self.nlights = f.value, m.value, n.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_scene_free(self.h)
            self.h = None

    def facets(self):
        F = self.nfacets
        v = np.zeros((F, 18), np.float32)
        mat = np.zeros(F, np.int32)
        lo = np.zeros(F, np.int32)
        un = np.zeros((F, 3), np.float64)
        lib().orc_scene_facets(self.h, v, mat, lo, un)
        return v, mat, lo, un

    def materials(self):
        m = np.zeros((self.nmaterials, 7), np.float32)
        lib().orc_scene_materials(self.h, m)
        return m

    def lights(self):
        f = np.zeros(self.nlights, np.int32)
        a = np.zeros((self.nlights, 4), np.float64)
        lib().orc_scene_lights(self.h, f, a)
        return f, a

    def camera(self):
        """the XML <camera> (dist_scale 1), or None if the file has none"""
        c = Camera()
        return c if lib().orc_scene_camera(self.h, C.byref(c)) == 0 else None

    def build_grid(self, camera_pos, n0=100000):
        lib().orc_grid_build(self.h, _v(camera_pos), n0)

    def grid_info(self):
        o = np.zeros(7)
        lib().orc_grid_info(self.h, o)
        return o

    def closest_hit(self, ro, rd, exclude=-1, light_only=False):
        tbg = np.zeros(3)
        fn = lib().orc_closest_light_hit if light_only else lib().orc_closest_hit
        f = fn(self.h, _v(ro), _v(rd), int(exclude), tbg)
        return f, tbg

    def light_prep(self, x1, n):
        cnt = C.c_int()
        idx = np.zeros(self.nlights + 1, np.int32)
        w = np.zeros(self.nlights + 1)
        ws = lib().orc_light_prep(self.h, _v(x1), _v(n), C.byref(cnt), idx, w)
        return ws, idx[:cnt.value], w[:cnt.value]

    def light_sample_ref(self, ctr, x1, n):
        o = np.zeros(6)
        lib().orc_light_sample_ref(self.h, int(ctr), _v(x1), _v(n), o)
        return o

    def light_sample_u(self, x1, n, u, xi1, xi2):
        o = np.zeros(6)
        lib().orc_light_sample_u(self.h, _v(x1), _v(n), u, xi1, xi2, o)
        return o

    def light_pdf(self, x1, n, facet):
        return lib().orc_light_pdf(self.h, _v(x1), _v(n), int(facet))

    def shade_sample(self, cam, mode, rng, key, i, j, sample=0):
        rgb = np.zeros(3)
        draws = C.c_uint64()
        lib().orc_shade_sample(self.h, C.byref(cam), mode, rng, int(key), i, j, sample, rgb, C.byref(draws))
        return rgb, draws.value

    def render(self, cam, mode, seed, spp, s0=0, s1=None, stride=1, offset=0, nthreads=1, out=None):
        if s1 is None:
            s1 = spp
        if out is None:
            out = np.zeros((cam.height, cam.width, 3))
        stats = np.zeros(4, np.uint64)
        rc = lib().orc_render(self.h, C.byref(cam), mode, int(seed), spp, s0, s1, stride, offset, nthreads,
                              out.reshape(-1), stats)
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return out, stats

    def depth_study(self, cam, seed, spp, max_depth, stride=1, offset=0, nthreads=1):
        """MIS frame with the tree cut below depth max_depth (<= 62) and the nodes per depth (64 counts, [63] =
        nodes cut by the cap): orc_depth_study"""
        out = np.zeros((cam.height, cam.width, 3))
        hist = np.zeros(64, np.uint64)
        rc = lib().orc_depth_study(self.h, C.byref(cam), int(seed), spp, stride, offset, nthreads, int(max_depth),
                                   out.reshape(-1), hist)
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return out, hist


def brdf_phong(n, wi, wr, kd, ks, ns):
    o = np.zeros(3)
    lib().orc_brdf_phong(_v(n), _v(wi), _v(wr), _v(kd), _v(ks), ns, o)
    return o


def phong_pdf(n, wi, wr, kd, ks, ns):
    return lib().orc_phong_pdf(_v(n), _v(wi), _v(wr), _v(kd), _v(ks), ns)


def sample_phong_ref(ctr, n, wr, kd, ks, ns):
    o = np.zeros(4)
    lib().orc_sample_phong_ref(int(ctr), _v(n), _v(wr), _v(kd), _v(ks), ns, o)
    return o


def tone_map(rgb, maxr=380.0, gamma=0.25):
    o = np.zeros(3, np.int32)
    lib().orc_tone_map(_v(rgb), maxr, gamma, o)
    return o


def camera_ray(cam, i, j):
    e, d = np.zeros(3), np.zeros(3)
    lib().orc_camera_ray(C.byref(cam), i, j, e, d)
    return e, d


def counter_uniform(seed, pixel, sample, node, dim):
    return lib().orc_counter_uniform(seed, pixel, sample, node, dim)
