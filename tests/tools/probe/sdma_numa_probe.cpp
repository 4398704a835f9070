// SDMA device -> pinned host copy rate by the CPU agent passed as the
// destination agent, and which agent owns a hipHostMalloc buffer (two-socket
// hosts: the code-stream D2H of GpuEncoder::dma_to_host).
//   hipcc --offload-arch=gfx950 -O2 sdma_numa_probe.cpp -lhsa-runtime64 -o sdma_numa_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static hsa_status_t cpus(hsa_agent_t a, void *d) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU) ((std::vector<hsa_agent_t> *)d)->push_back(a);
    return HSA_STATUS_SUCCESS;
}

int main() {
    const size_t n = 342ull << 20;
    hipSetDevice(0);
    uint8_t *d = nullptr, *h = nullptr;
    hipMalloc(&d, n);
    hipHostMalloc((void **)&h, n, hipHostMallocDefault);
    hipMemset(d, 1, n);
    memset(h, 0, n);
    hipDeviceSynchronize();
    std::vector<hsa_agent_t> cpu;
    hsa_iterate_agents(cpus, &cpu);
    hsa_amd_pointer_info_t pi;
    memset(&pi, 0, sizeof pi);
    pi.size = sizeof pi;
    hsa_amd_pointer_info(d, &pi, nullptr, nullptr, nullptr);
    hsa_agent_t gpu = pi.agentOwner;
    memset(&pi, 0, sizeof pi);
    pi.size = sizeof pi;
    hsa_amd_pointer_info(h, &pi, nullptr, nullptr, nullptr);
    hsa_device_type_t ot;
    hsa_agent_get_info(pi.agentOwner, HSA_AGENT_INFO_DEVICE, &ot);
    int owner = -1;
    for (size_t i = 0; i < cpu.size(); i++) if (cpu[i].handle == pi.agentOwner.handle) owner = (int)i;
    printf("cpu agents %zu; pinned buffer owner: type %d, cpu index %d\n", cpu.size(), (int)ot, owner);
    hsa_signal_t sig;
    hsa_signal_create(1, 0, nullptr, &sig);
    hipStream_t s;
    hipStreamCreate(&s);
    uint32_t mask = 0, rec = 0;
    hsa_amd_memory_copy_engine_status(cpu[0], gpu, &mask);
    hsa_amd_memory_get_preferred_copy_engine(cpu[0], gpu, &rec);
    printf("engines: available 0x%x recommended 0x%x\n", mask, rec);
    for (int e = 0; e < 16; e++) {
        if (!(mask & (1u << e))) continue;
        double best = 0;
        for (int r = 0; r < 2; r++) {
            hsa_signal_store_relaxed(sig, 1);
            const double t0 = now();
            if (hsa_amd_memory_async_copy_on_engine(h, cpu[0], d, gpu, n, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)(1u << e), true) != HSA_STATUS_SUCCESS) { printf("engine %d: refused\n", e); break; }
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            const double g = n / (now() - t0) / 1e9;
            best = g > best ? g : best;
        }
        printf("engine %2d: %.2f GB/s\n", e, best);
    }
    for (int rep = 0; rep < 2; rep++) {
        for (size_t i = 0; i < cpu.size(); i++) {
            hsa_signal_store_relaxed(sig, 1);
            const double t0 = now();
            hsa_amd_memory_async_copy(h, cpu[i], d, gpu, n, 0, nullptr, sig);
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            printf("sdma, dst agent cpu %zu: %.2f GB/s\n", i, n / (now() - t0) / 1e9);
        }
        hsa_signal_store_relaxed(sig, 1);
        double t0 = now();
        hsa_amd_memory_async_copy(h, pi.agentOwner, d, gpu, n, 0, nullptr, sig);
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        printf("sdma, dst agent = owner: %.2f GB/s\n", n / (now() - t0) / 1e9);
        hsa_signal_store_relaxed(sig, 1);
        t0 = now();
        hsa_amd_memory_async_copy(h, gpu, d, gpu, n, 0, nullptr, sig);
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        printf("copy, both agents gpu: %.2f GB/s\n", n / (now() - t0) / 1e9);
        t0 = now();
        hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        printf("blit: %.2f GB/s\n", n / (now() - t0) / 1e9);
    }
    return 0;
}
