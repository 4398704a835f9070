// Dependent-issue latencies on gfx950 that bound the MQ coder's per-decision
// chains (t1.hip k_t1_mq): cycles per dependent VALU op, per VALU->VCC->
// cndmask hop, per dependent LDS read, for one wave alone on its SIMD.
//   hipcc --offload-arch=gfx950 -O3 latency_probe.hip -o latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void dep_add(unsigned *out, unsigned long long *cyc, int iters) {
    unsigned x = threadIdx.x;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) asm volatile("v_add_u32 %0, %0, 7" : "+v"(x));
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// two independent chains interleaved
__global__ void dep_add2(unsigned *out, unsigned long long *cyc, int iters) {
    unsigned x = threadIdx.x, y = threadIdx.x * 3;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            asm volatile("v_add_u32 %0, %0, 7" : "+v"(x));
            asm volatile("v_add_u32 %0, %0, 5" : "+v"(y));
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = x + y;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// four independent chains interleaved
__global__ void dep_add4(unsigned *out, unsigned long long *cyc, int iters) {
    unsigned x = threadIdx.x, y = threadIdx.x * 3, z = threadIdx.x * 5, w = threadIdx.x * 7;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            asm volatile("v_add_u32 %0, %0, 7" : "+v"(x));
            asm volatile("v_add_u32 %0, %0, 5" : "+v"(y));
            asm volatile("v_add_u32 %0, %0, 3" : "+v"(z));
            asm volatile("v_add_u32 %0, %0, 1" : "+v"(w));
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = x + y + z + w;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// compare -> vcc -> cndmask chain (a select whose condition comes from the previous value)
__global__ void dep_cmp_sel(unsigned *out, unsigned long long *cyc, int iters) {
    unsigned x = threadIdx.x;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++)
            asm volatile("v_cmp_lt_u32 vcc, 100, %0\n v_cndmask_b32 %0, 3, %0, vcc" : "+v"(x) : : "vcc");
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// VALU -> SGPR pair -> SALU and -> VALU use
__global__ void dep_cmp_salu(unsigned *out, unsigned long long *cyc, int iters) {
    unsigned x = threadIdx.x;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++)
            asm volatile("v_cmp_lt_u32 vcc, 100, %0\n v_cmp_ne_u32 s[4:5], 7, %0\n s_and_b64 vcc, s[4:5], vcc\n v_addc_co_u32 %0, vcc, 0, %0, vcc"
                         : "+v"(x) : : "vcc", "s4", "s5");
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// dependent LDS reads (pointer chase through LDS)
__global__ void dep_lds(unsigned *out, unsigned long long *cyc, int iters) {
    __shared__ unsigned tab[64 * 64];
    for (int i = threadIdx.x; i < 64 * 64; i += 64) tab[i] = ((i + 64 * 7) & (64 * 64 - 1));
    __syncthreads();
    unsigned x = threadIdx.x;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) x = tab[x];
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    unsigned *out;
    unsigned long long *cyc, h[4096];
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cyc, 8 * 4096);
    const int iters = 4096;
    struct { const char *name; void (*k)(unsigned *, unsigned long long *, int); double per; } ks[] = {
        {"dependent v_add_u32", dep_add, 16.0}, {"two interleaved v_add chains (per op)", dep_add2, 32.0},
        {"v_cmp->vcc->v_cndmask hop", dep_cmp_sel, 16.0}, {"v_cmp x2 -> s_and -> v_addc hop", dep_cmp_salu, 16.0},
        {"dependent ds_read_b32", dep_lds, 16.0}, {"four interleaved v_add chains (per op)", dep_add4, 64.0}};
    {   // calibrate the counter: one wave of dep_add timed by events
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipLaunchKernelGGL(dep_add, dim3(1), dim3(64), 0, 0, out, cyc, iters * 8);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(dep_add, dim3(1), dim3(64), 0, 0, out, cyc, iters * 8);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
        printf("counter: %llu ticks in %.3f ms -> %.1f MHz\n", h[0], ms, h[0] / (ms * 1e3));
    }
    for (auto &k : ks) {
        for (int waves : {1, 256, 1024, 4096}) {  // one per SIMD at most .. 4 per SIMD
            hipLaunchKernelGGL(k.k, dim3(waves), dim3(64), 0, 0, out, cyc, iters);
            hipDeviceSynchronize();
            hipMemcpy(h, cyc, 8 * (waves < 1024 ? waves : 1024), hipMemcpyDeviceToHost);
            double s = 0; int n = waves < 1024 ? waves : 1024;
            for (int i = 0; i < n; i++) s += h[i];
            printf("%-40s waves %5d: %6.2f cycles per op\n", k.name, waves, s / n / (iters * k.per));
        }
    }
    return 0;
}
