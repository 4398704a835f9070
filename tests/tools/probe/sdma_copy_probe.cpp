// Device -> pinned-host copy engines on MI355X: the HIP runtime's copy
// (hipMemcpyAsync, a __amd_rocclr_copyBuffer blit kernel on the CUs for
// pinned memory) against ROCr's DMA path (hsa_amd_memory_async_copy, SDMA
// engines), alone and next to a kernel that occupies every CU.
//   hipcc --offload-arch=gfx950 -O2 sdma_copy_probe.cpp -lhsa-runtime64 -o sdma_copy_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char *m_ = ""; hsa_status_string(s_, &m_); printf("%s: %s\n", #x, m_); return 1; } } while (0)

__global__ void busy(float *out, int iters) {
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    for (int i = 0; i < iters; i++) a = a * b + 1e-7f;
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

__global__ void fill(uint8_t *d, size_t n, uint8_t v) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += (size_t)gridDim.x * blockDim.x)
        ((uint32_t *)d)[i] = 0x01010101u * v;
}
// releases a copy waiting on `dep`: the stream's earlier kernels are done
__global__ void release_dep(int64_t *dep) {
    __hip_atomic_store(dep, (int64_t)0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static hsa_status_t find_cpu(hsa_agent_t a, void *d) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU) { *(hsa_agent_t *)d = a; return HSA_STATUS_INFO_BREAK; }
    return HSA_STATUS_SUCCESS;
}

int main() {
    const size_t n = 256ull << 20;
    CK(hipSetDevice(0));
    uint8_t *d = nullptr, *h = nullptr;
    float *bo = nullptr;
    CK(hipMalloc(&d, n));
    CK(hipMalloc(&bo, 4096 * 256 * 4));
    CK(hipHostMalloc((void **)&h, n, hipHostMallocDefault));
    CK(hipMemset(d, 0x5A, n));
    CK(hipDeviceSynchronize());
    hipStream_t s, sb;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hsa_amd_pointer_info_t pi;
    std::memset(&pi, 0, sizeof pi);
    pi.size = sizeof pi;
    HK(hsa_amd_pointer_info(d, &pi, nullptr, nullptr, nullptr));
    hsa_agent_t gpu = pi.agentOwner, cpu{0};
    HK(hsa_iterate_agents(find_cpu, &cpu) == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR);
    uint32_t mask = 0, rec = 0;
    hsa_amd_memory_copy_engine_status(cpu, gpu, &mask);
    hsa_amd_memory_get_preferred_copy_engine(cpu, gpu, &rec);
    printf("sdma engines gpu->cpu: available mask 0x%x, recommended 0x%x\n", mask, rec);
    hsa_signal_t sig;
    HK(hsa_signal_create(1, 0, nullptr, &sig));
    auto sdma = [&](size_t bytes) -> int {
        hsa_signal_store_relaxed(sig, 1);
        HK(hsa_amd_memory_async_copy(h, cpu, d, gpu, bytes, 0, nullptr, sig));
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        return 0;
    };
    auto blit = [&](size_t bytes) -> int {
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        return 0;
    };
    // multi-engine: the copy cut into k pieces on the recommended engines
    std::vector<hsa_signal_t> sigs(8);
    for (auto &x : sigs) HK(hsa_signal_create(1, 0, nullptr, &x));
    auto sdma_k = [&](size_t bytes, int k) -> int {
        int eng[8], ne = 0;
        for (int b = 0; b < 16 && ne < k; b++) if (mask & (1u << b)) eng[ne++] = b;
        if (ne == 0) return 1;
        const size_t piece = (bytes / ne + 4095) & ~(size_t)4095;
        for (int i = 0; i < ne; i++) {
            const size_t o = i * piece, m = o >= bytes ? 0 : (bytes - o < piece ? bytes - o : piece);
            hsa_signal_store_relaxed(sigs[i], 1);
            if (!m) { hsa_signal_store_relaxed(sigs[i], 0); continue; }
            HK(hsa_amd_memory_async_copy_on_engine(h + o, cpu, d + o, gpu, m, 0, nullptr, sigs[i],
                                                   (hsa_amd_sdma_engine_id_t)(1u << eng[i]), true));
        }
        for (int i = 0; i < ne; i++)
            hsa_signal_wait_scacquire(sigs[i], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        return 0;
    };
    {   // chained: the copy is queued first and waits on a signal a kernel releases
        hsa_signal_t dep;
        HK(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &dep));
        volatile hsa_signal_value_t *dv = nullptr;
        HK(hsa_amd_signal_value_pointer(dep, &dv));
        int bad = 0;
        double tsum = 0;
        for (int it = 0; it < 20; it++) {
            const uint8_t v = (uint8_t)(it * 37 + 11);
            hsa_signal_store_relaxed(dep, 1);
            hsa_signal_store_relaxed(sig, 1);
            const double t0 = now();
            hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, d, n, v);
            hipLaunchKernelGGL(release_dep, dim3(1), dim3(1), 0, s, (int64_t *)dv);
            CK(hipGetLastError());
            HK(hsa_amd_memory_async_copy(h, cpu, d, gpu, n, 1, &dep, sig));
            if (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 10000000000ull, HSA_WAIT_STATE_BLOCKED) != 0) {
                printf("chained copy: timed out\n");
                return 1;
            }
            tsum += now() - t0;
            for (size_t i = 0; i < n; i += 4093) bad += h[i] != v;
            bad += h[n - 1] != v;
            CK(hipStreamSynchronize(s));
        }
        printf("chained (kernel releases the SDMA copy): %s, %.2f GB/s incl. the fill\n", bad ? "DATA WRONG" : "data ok",
               20.0 * n / tsum / 1e9);
    }
    for (int rep = 0; rep < 2; rep++) {
        for (int mode = 0; mode < 4; mode++) {
            const char *name[] = {"blit (hipMemcpyAsync)", "sdma (hsa_amd_memory_async_copy)", "sdma x2 engines", "sdma x4 engines"};
            for (int load = 0; load < 2; load++) {
                if (load) {  // every CU busy for ~the copy's duration
                    hipLaunchKernelGGL(busy, dim3(4096), dim3(256), 0, sb, bo, 2000000);
                    CK(hipGetLastError());
                }
                std::memset(h, 0, 4096);
                const double t0 = now();
                int r = 0;
                for (int i = 0; i < 4 && !r; i++)
                    r = mode == 0 ? blit(n) : mode == 1 ? sdma(n) : sdma_k(n, mode == 2 ? 2 : 4);
                const double dt = now() - t0;
                if (r) { printf("%s failed\n", name[mode]); continue; }
                const bool ok = h[0] == 0x5A && h[n - 1] == 0x5A;
                printf("%-36s %-10s %7.2f GB/s %s\n", name[mode], load ? "CUs busy" : "idle", 4.0 * n / dt / 1e9, ok ? "" : "DATA WRONG");
                CK(hipStreamSynchronize(sb));
            }
        }
    }
    return 0;
}
