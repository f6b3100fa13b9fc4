"""Counter-based RNG of the GPU path (csrc/device_math.h counter_key / counter_u), in Python.

Keyed by (seed, pixel, sample, node, dim): node = heap id in the MIS tree (root 1, light child
2n, BRDF child 2n+1) or depth+1 on a BRDF-only path; dims 0 RR, 1 light pick, 2-3 Arvo xi1/xi2,
4 lobe pick, 5-6 lobe xi1/xi2.  Replaces the reference's clock-seeded std::default_random_engine
per RNG site (main.cpp:431-434, BRDF.cpp:38-39, Mylight.cpp:432-433), which is not reproducible.
"""
M64 = (1 << 64) - 1


def mix64(z):
    z &= M64
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return z


def counter_key(seed, pixel, sample, node):
    k = mix64(seed + 0x9E3779B97F4A7C15 * (pixel + 1))
    k = mix64(k ^ ((0xD1B54A32D192ED03 * (sample + 1)) & M64))
    return mix64(k ^ ((0xA24BAED4963EE407 * node) & M64))


def counter_u(key, dim):
    return (mix64(key + 0x9FB21C651E98DF25 * (dim + 1)) >> 11) * 2.0 ** -53


def counter_uniform(seed, pixel, sample, node, dim):
    return counter_u(counter_key(seed, pixel, sample, node), dim)
