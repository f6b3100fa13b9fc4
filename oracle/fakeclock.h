// TEST INFRASTRUCTURE ONLY (oracle/_ref build).  Force-included (-include) into every reference
// translation unit compiled by oracle/Makefile so that the reference's clock-seeded RNG sites
// (main.cpp:431-434, BRDF.cpp:38-39, Mylight.cpp:432-433, ...) become
// deterministic.  `std::chrono::system_clock::now()` is redirected to a counter hashed with
// splitmix64 (a multiplicative counter correlates the per-call reseeded minstd_rand0 streams and
// biases MIS).  The oracle's RefRng (oracle/mcpt_oracle.c) replays exactly
// this seed sequence.  Nothing here is shipped or linked into the product.
#pragma once
#include <chrono>

namespace std {
namespace chrono {
struct mcpt_fake_clock {
    static inline unsigned long long ctr = 0;
    static system_clock::time_point now() {
        unsigned long long z = (++ctr) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        return system_clock::time_point(system_clock::duration((long long)(z >> 1)));
    }
};
}  // namespace chrono
}  // namespace std
#define system_clock mcpt_fake_clock
