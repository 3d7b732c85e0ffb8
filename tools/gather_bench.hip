// Microbenchmark: the cost model of the BVH node fetch on MI355X.
// Every lane walks a dependent chain through a table of 64-B "nodes"; the
// next index comes from the loaded data, as in a traversal step.
//   mode 0..3 : 1/2/4 dwordx4 or 4 dword loads per step from global memory
//   mode 4    : 4 x ds_read_b128 from a 32 KB LDS table
// Lanes are grouped: `group` consecutive lanes share a node (1 = fully
// divergent, 64 = one node per wave).  Prints cycles per wave-step (s_memtime)
// and wave-steps per CU-cycle.
//   hipcc --offload-arch=gfx950 -O3 tools/gather_bench.hip -o tools/gather_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) (void)(x)

struct alignas(16) F4 {
    float x, y, z, w;
};

template <int MODE>
__global__ void chase(const F4 *__restrict__ nodes, unsigned n_nodes, int steps, int group,
                      unsigned long long *cycles, float *sink) {
    __shared__ F4 tab[2048];                 // 32 KB: 512 nodes of 64 B
    if (MODE == 4) {
        for (int i = threadIdx.x; i < 2048; i += blockDim.x) tab[i] = nodes[i];
        __syncthreads();
        n_nodes = 512;
    }
    unsigned lane = threadIdx.x & 63;
    unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    unsigned g = lane / group;               // lanes of a group share a node
    unsigned salt = g * 97u;
    unsigned idx = ((wave * 64 + g) * 2654435761u) % n_nodes;
    float acc = 0.0f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; s++) {
        unsigned nxt;
        if (MODE == 4) {
            const F4 *N = tab + 4 * idx;
            F4 a = N[0], b = N[1], c = N[2], d = N[3];
            acc += a.x + b.y + c.z;
            nxt = __float_as_uint(d.w);
        } else if (MODE == 3) {
            const float *N = reinterpret_cast<const float *>(nodes + 4 * (size_t)idx);
            float a = N[0], b = N[5], c = N[10], d = N[15];
            acc += a + b + c;
            nxt = __float_as_uint(d);
        } else {
            const F4 *N = nodes + 4 * (size_t)idx;
            F4 d = N[3];
            if (MODE >= 1) {
                F4 c = N[2];
                acc += c.z;
            }
            if (MODE >= 2) {
                F4 a = N[0], b = N[1];
                acc += a.x + b.y;
            }
            nxt = __float_as_uint(d.w);
        }
        idx = (nxt ^ salt) % n_nodes;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) atomicAdd(cycles, t1 - t0);
    if (acc == 12345.0f) sink[0] = acc;
}

typedef void (*KFn)(const F4 *, unsigned, int, int, unsigned long long *, float *);

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned long long *dcyc;
    float *sink;
    CHECK(hipMalloc(&dcyc, sizeof(unsigned long long)));
    CHECK(hipMalloc(&sink, sizeof(float)));
    unsigned n_nodes = 64 * 1024 / 64;       // 64 KB table (L2-resident, 2x L1)
    std::vector<F4> h((size_t)n_nodes * 4);
    for (size_t i = 0; i < h.size(); i++) {
        unsigned r = (unsigned)(i * 2246822519u + 12345u);
        float f;
        memcpy(&f, &r, sizeof f);
        h[i] = {1.0f, 2.0f, 3.0f, f};
    }
    F4 *d;
    CHECK(hipMalloc(&d, h.size() * sizeof(F4)));
    CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(F4), hipMemcpyHostToDevice));
    KFn fns[5] = {chase<0>, chase<1>, chase<2>, chase<3>, chase<4>};
    const char *names[5] = {"1 x dwordx4", "2 x dwordx4", "4 x dwordx4", "4 x dword", "4 x ds_read_b128"};
    printf("CUs %d, 20 waves/CU\n", cus);
    for (int m = 0; m < 5; m++)
        for (int group : {1, 2, 4, 8, 16, 64}) {
            int wpc = 20, blocks = cus * wpc / 4, steps = 1000;
            hipLaunchKernelGGL(fns[m], dim3(blocks), dim3(256), 0, 0, d, n_nodes, 20, group, dcyc, sink);
            CHECK(hipMemset(dcyc, 0, sizeof(unsigned long long)));
            hipEvent_t e0, e1;
            CHECK(hipEventCreate(&e0));
            CHECK(hipEventCreate(&e1));
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(fns[m], dim3(blocks), dim3(256), 0, 0, d, n_nodes, steps, group, dcyc, sink);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            unsigned long long cyc = 0;
            CHECK(hipMemcpy(&cyc, dcyc, sizeof cyc, hipMemcpyDeviceToHost));
            double waves = blocks * 4.0;
            double per_step = (double)cyc / waves / steps;
            double cu_cycles_per_wavestep = (ms * 1e-3 * 2.4e9) * cus / (waves * steps);
            printf("%-18s lanes/node %2d  cycles/step %6.0f  CU-cycles per wave-step %6.1f\n", names[m], group,
                   per_step, cu_cycles_per_wavestep);
            CHECK(hipEventDestroy(e0));
            CHECK(hipEventDestroy(e1));
        }
    return 0;
}
