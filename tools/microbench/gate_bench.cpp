// gate_bench.cpp — host time of the key-dedupe gate (cv_api.cpp dedupe_gate), which every large
// cv_ed25519_verify_batch call runs before its first DMA, on 1M / 8M distinct keys and on keys repeated 8 times
// in a row, with the keys evicted from the caches before each call (a fresh call's state).  No GPU needed: the
// engine's translation unit is included for its host code only and the kernel symbols are left unresolved.
//   /opt/rocm/bin/hipcc -x hip --offload-host-only -O3 -std=c++17 -Iinclude -Icorda_amd/csrc \
//       tools/microbench/gate_bench.cpp -o /tmp/gate_bench -lpthread -Wl,--unresolved-symbols=ignore-all
#include "../../corda_amd/csrc/cv_api.cpp"

#include <chrono>
#include <random>

int main() {
    static std::vector<uint8_t> junk(64 << 20);
    for (size_t n : {1000000ul, 8000000ul}) {
        std::vector<uint8_t> pk(n * 32), pk8(n * 32);
        std::mt19937_64 g(1);
        for (auto &x : pk) x = (uint8_t)g();
        for (size_t i = 0; i < n; i++) std::memcpy(&pk8[32 * i], &pk[32 * (i / 8)], 32);
        double best = 1e9, sum = 0;
        int yes = 0, yes8 = 0;
        const int reps = 40;
        for (int r = 0; r < reps; r++) {
            for (size_t q = 0; q < junk.size(); q += 64) junk[q]++;   // evict the keys
            const auto t0 = std::chrono::steady_clock::now();
            yes += dedupe_gate(n, pk.data());
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            best = std::min(best, dt);
            sum += dt;
            yes8 += dedupe_gate(n, pk8.data());
        }
        std::printf("n=%zu gate min %.1f us mean %.1f us; keyed: distinct %d/%d, 8x repeated %d/%d\n", n, best * 1e6,
                    sum / reps * 1e6, yes, reps, yes8, reps);
    }
    return 0;
}
