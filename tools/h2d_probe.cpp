// Host<->device transfer probe for the host-staged entry points (gasalx_align_host):
// pageable vs registered vs pinned-staging copies of a config-2-sized batch.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static void pmemcpy(char *d, const char *s, size_t n, int t) {
    std::vector<std::thread> th;
    size_t per = (n + t - 1) / t;
    for (int i = 0; i < t; i++) {
        size_t a = i * per, b = std::min(n, a + per);
        if (a < b) th.emplace_back([=] { std::memcpy(d + a, s + a, b - a); });
    }
    for (auto &x : th) x.join();
}

int main(int argc, char **argv) {
    size_t n = (argc > 1 ? atol(argv[1]) : 320) << 20;
    char *h = (char *)malloc(n);
    memset(h, 1, n);
    void *d; CK(hipMalloc(&d, n));
    hipStream_t st; CK(hipStreamCreate(&st));
    CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));   // warm
    double t = now(); CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice)); double pageable = now() - t;
    t = now(); CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost)); double pageable_d2h = now() - t;
    t = now(); CK(hipHostRegister(h, n, hipHostRegisterDefault)); double reg = now() - t;
    t = now(); CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st)); double regcp = now() - t;
    t = now(); CK(hipHostUnregister(h)); double unreg = now() - t;
    char *p; CK(hipHostMalloc((void **)&p, n, 0));
    memset(p, 2, n);
    t = now(); CK(hipMemcpyAsync(d, p, n, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st)); double pin = now() - t;
    t = now(); CK(hipMemcpyAsync(p, d, n, hipMemcpyDeviceToHost, st)); CK(hipStreamSynchronize(st)); double pin_d2h = now() - t;
    double mc[4]; int thr[4] = {1, 4, 8, 16};
    for (int i = 0; i < 4; i++) { t = now(); pmemcpy(p, h, n, thr[i]); mc[i] = now() - t; }
    double gb = n / 1e9;
    printf("{\"bytes\": %zu, \"pageable_h2d_GBs\": %.2f, \"pageable_d2h_GBs\": %.2f, \"register_ms\": %.2f, "
           "\"registered_h2d_GBs\": %.2f, \"unregister_ms\": %.2f, \"pinned_h2d_GBs\": %.2f, \"pinned_d2h_GBs\": %.2f, "
           "\"memcpy_GBs\": {\"1\": %.2f, \"4\": %.2f, \"8\": %.2f, \"16\": %.2f}, \"hw_threads\": %u}\n",
           n, gb / pageable, gb / pageable_d2h, reg * 1e3, gb / regcp, unreg * 1e3, gb / pin, gb / pin_d2h,
           gb / mc[0], gb / mc[1], gb / mc[2], gb / mc[3], std::thread::hardware_concurrency());
    return 0;
}
