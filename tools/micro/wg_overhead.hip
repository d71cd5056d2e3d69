// Microbenchmark: cost of a 4096-workgroup launch whose workgroups do almost nothing (read one word,
// write one word per thread, like the raster's "nothing" ablation) vs the same work done by a persistent
// grid looping over the 4096 tiles.  Build: hipcc --offload-arch=gfx950 -O3 -o wg_overhead wg_overhead.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(256) void per_tile(const unsigned *counts, int *out, int ntx)
{
    const int tile = blockIdx.x, t = threadIdx.x;
    const int tx = tile % ntx, ty = tile / ntx;
    const unsigned c = counts[tile & 255];
    const int i = tx * 16 + (t & 15), j = ty * 16 + (t >> 4);
    out[j * ntx * 16 + i] = (int)c + t;
}

__global__ __launch_bounds__(256) void persistent(const unsigned *counts, int *out, int ntx, int ntiles)
{
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int t = threadIdx.x;
        const int tx = tile % ntx, ty = tile / ntx;
        const unsigned c = counts[tile & 255];
        const int i = tx * 16 + (t & 15), j = ty * 16 + (t >> 4);
        out[j * ntx * 16 + i] = (int)c + t;
    }
}

int main()
{
    const int ntx = 64, ntiles = 4096;
    unsigned *counts; int *out;
    hipMalloc(&counts, 1024); hipMemset(counts, 0, 1024);
    hipMalloc(&out, 1024 * 1024 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    auto time = [&](auto launch) {
        for (int w = 0; w < 20; ++w) launch();
        std::vector<float> v;
        for (int r = 0; r < 50; ++r) {
            hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); v.push_back(ms * 1e3f);
        }
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    printf("per-tile 4096 WGs           %.2f us\n", time([&] { per_tile<<<ntiles, 256>>>(counts, out, ntx); }));
    for (int g : {256, 512, 1024, 1792, 2048})
        printf("persistent %4d WGs         %.2f us\n", g, time([&] { persistent<<<g, 256>>>(counts, out, ntx, ntiles); }));
    printf("empty 1-WG launch           %.2f us\n", time([&] { persistent<<<1, 64>>>(counts, out, ntx, 0); }));
    return 0;
}
