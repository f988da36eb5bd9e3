// ptr_attr.cpp — host cost of hipPointerGetAttributes (the engine's pinned-input test, cv_api.cpp host_pinned) on
// pinned and pageable pointers, with few and with many live pinned allocations, and while another thread waits in
// hipEventSynchronize on a long kernel (lock contention).
//   hipcc -O2 ptr_attr.cpp -o ptr_attr && ./ptr_attr
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

__global__ void spin(unsigned long long cycles, int *out) {
    const unsigned long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

static double per_call_us(const void *p, int reps) {
    hipPointerAttribute_t a;
    const double t0 = now();
    for (int i = 0; i < reps; i++) (void)hipPointerGetAttributes(&a, static_cast<const char *>(p) + (i & 1023));
    (void)hipGetLastError();
    return (now() - t0) / reps * 1e6;
}

int main() {
    const size_t big = 64 << 20;
    void *pinned = nullptr;
    if (hipHostMalloc(&pinned, big, hipHostMallocDefault) != hipSuccess) return 1;
    std::vector<char> pageable(big);
    const int reps = 20000;
    printf("pinned, 1 live pinned allocation:    %.3f us per call\n", per_call_us(pinned, reps));
    printf("pageable, 1 live pinned allocation:  %.3f us per call\n", per_call_us(pageable.data(), reps));
    std::vector<void *> many;
    for (int i = 0; i < 2000; i++) {
        void *q = nullptr;
        if (hipHostMalloc(&q, 1 << 20, hipHostMallocDefault) != hipSuccess) break;
        many.push_back(q);
    }
    printf("pinned, %zu live pinned allocations: %.3f us per call\n", many.size() + 1, per_call_us(pinned, reps));
    printf("pageable, %zu live:                  %.3f us per call\n", many.size() + 1, per_call_us(pageable.data(), reps));
    for (void *q : many) (void)hipHostFree(q);
    many.clear();
    printf("pinned, after freeing them:          %.3f us per call\n", per_call_us(pinned, reps));
    // another thread blocked in hipEventSynchronize on a ~200 ms kernel
    int *flag = nullptr;
    (void)hipMalloc(&flag, 4);
    hipEvent_t ev;
    (void)hipEventCreate(&ev);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 200ull * 1000 * 1000 * 2, flag);
    (void)hipEventRecord(ev, s);
    std::atomic<bool> waiting{false};
    std::thread th([&] {
        waiting = true;
        (void)hipEventSynchronize(ev);
    });
    while (!waiting) {
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    printf("pinned, another thread in hipEventSynchronize: %.3f us per call\n", per_call_us(pinned, 2000));
    th.join();
    (void)hipStreamSynchronize(s);
    (void)hipFree(flag);
    (void)hipHostFree(pinned);
    return 0;
}
