// Microbenchmark: dependent random 64 B line gathers (pointer chasing) on MI355X.
// Each lane follows its own chain through a table of 64 B lines whose first word
// is the index of the next line.  Modes:
//   0  per-lane: 4 x global_load_dwordx4 of the lane's own line
//   1  per-lane: 1 x global_load_dword (only the link word)
//   2  cooperative: 4 lanes load one line (16 B each) through LDS, each lane then
//      reads its own 64 B back from LDS
// usage: gather <table MiB> <mode> <steps> <waves per SIMD (1..8)>
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_init(uint4* tab, uint64_t n, uint64_t mult, uint64_t add)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // a full-period LCG-like permutation step: next = (i * mult + add) mod n with n a power of 2
    const uint64_t nx = (i * mult + add) & (n - 1);
    tab[i * 4 + 0] = make_uint4((uint32_t)nx, (uint32_t)(nx >> 32), (uint32_t)i, 7u);
    tab[i * 4 + 1] = make_uint4(1, 2, 3, 4);
    tab[i * 4 + 2] = make_uint4(5, 6, 7, 8);
    tab[i * 4 + 3] = make_uint4(9, 10, 11, 12);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_chase(const uint4* __restrict__ tab, uint64_t n, int steps, uint64_t* out)
{
    __shared__ uint4 lds[4][64 * 4];   // per wave: 64 lines x 64 B
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t cur = (gid * 0x9E3779B97F4A7C15ull) & (n - 1);
    uint32_t acc = 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int s = 0; s < steps; ++s) {
        if (MODE == 0) {
            const uint4* p = tab + cur * 4;
            const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
            acc += a.z + b.x + c.y + d.w;
            cur = (uint64_t)a.x | ((uint64_t)a.y << 32);
        } else if (MODE == 1) {
            const uint2 a = *reinterpret_cast<const uint2*>(tab + cur * 4);
            acc += a.x;
            cur = (uint64_t)a.x | ((uint64_t)a.y << 32);
        } else {
            // cooperative: instruction k loads the lines of lanes 16k..16k+15, 4 lanes per line
            #pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int owner = 16 * k + (lane >> 2);
                const uint64_t oc = ((uint64_t)__shfl(cur >> 32, owner) << 32) | (uint32_t)__shfl((uint32_t)cur, owner);
                const uint4 v = tab[oc * 4 + (lane & 3)];
                lds[w][owner * 4 + (lane & 3)] = v;
            }
            __builtin_amdgcn_s_barrier();   // wave-local data; a wave barrier suffices for ordering here
            const uint4 a = lds[w][lane * 4 + 0], b = lds[w][lane * 4 + 1], c = lds[w][lane * 4 + 2], d = lds[w][lane * 4 + 3];
            acc += a.z + b.x + c.y + d.w;
            cur = (uint64_t)a.x | ((uint64_t)a.y << 32);
            __builtin_amdgcn_s_barrier();
        }
    }
    out[gid] = cur + acc;
}

int main(int argc, char** argv)
{
    const uint64_t mib = argc > 1 ? strtoull(argv[1], 0, 0) : 16384;
    const int mode = argc > 2 ? atoi(argv[2]) : 0;
    const int steps = argc > 3 ? atoi(argv[3]) : 200;
    const int wps = argc > 4 ? atoi(argv[4]) : 8;
    uint64_t n = 1;
    while (n * 64 * 2 <= mib << 20) n <<= 1;
    uint4* tab; uint64_t* out;
    CK(hipMalloc(&tab, n * 64));
    hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    const uint64_t threads = (uint64_t)cus * 4 * wps * 64;
    CK(hipMalloc(&out, threads * 8));
    k_init<<<(n + 255) / 256, 256>>>(tab, n, 6364136223846793005ull | 1ull, 1442695040888963407ull | 1ull);
    CK(hipDeviceSynchronize());
    const unsigned blocks = (unsigned)(threads / 256);
    auto run = [&]() {
        if (mode == 0) k_chase<0><<<blocks, 256>>>(tab, n, steps, out);
        else if (mode == 1) k_chase<1><<<blocks, 256>>>(tab, n, steps, out);
        else k_chase<2><<<blocks, 256>>>(tab, n, steps, out);
    };
    run();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    run();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double lines = (double)threads * steps;
    printf("table %.0f MiB mode %d waves/SIMD %d: %.3f ms, %.3g lines/s, %.0f GB/s at 64 B, per-lane latency %.2f us\n",
           n * 64.0 / (1 << 20), mode, wps, ms, lines / (ms * 1e-3), lines * 64 / (ms * 1e-3) / 1e9,
           ms * 1e3 / steps);
    return 0;
}
