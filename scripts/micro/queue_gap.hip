// Diagnostic: the idle gap between two dependent kernels on one stream, as the
// replay stream sees it (last block's end of launch i -> first block's start of
// launch i+1, realtime clock, 10 ns ticks), under the engine's queue setups:
//   plain      default-priority stream, kernels back to back
//   hiprio     high-priority stream
//   wait       + a wait on an event of another stream that completed long ago
//   bound      + the waited event bound to the other stream's kernel, each
//              launch's stop event bound and waited on by a third stream
//   masked     + CU-masked other streams (as the engine's front / tail)
//   write      + each launch writes 10 MB (dirty L2 at its end)
// usage: queue_gap [launches]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ __launch_bounds__(512) void k_spin(uint64_t ticks, unsigned long long* st, unsigned long long* en, int i,
                                              double* out, size_t nw) {
    extern __shared__ double lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) atomicMin(&st[i], (unsigned long long)t0);
    lds[threadIdx.x] = (double)t0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    }
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < nw; k += (size_t)gridDim.x * blockDim.x)
        out[k] = (double)k + lds[threadIdx.x & 7];
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&en[i], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

__global__ void k_short(double* out) { out[threadIdx.x] = threadIdx.x; }

int main(int argc, char** argv) {
    const int L = argc > 1 ? atoi(argv[1]) : 24;
    const int grid = 96, block = 512;
    const size_t lds = 128 * 1024;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_spin), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    unsigned long long *st, *en;
    CK(hipMalloc(&st, 8 * L));
    CK(hipMalloc(&en, 8 * L));
    double *out, *aux;
    const size_t nw_big = 10u << 20 >> 3;
    CK(hipMalloc(&out, 8 * nw_big));
    CK(hipMalloc(&aux, 8 * 1024));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; c++)
        if (c % 32 != 31) mask[c / 32] |= 1u << (c % 32);
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    const char* names[] = {"plain", "hiprio", "wait", "bound", "masked", "write"};
    for (int v = 0; v < 6; v++) {
        hipStream_t c, f, t;
        if (v == 0)
            CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
        else
            CK(hipStreamCreateWithPriority(&c, hipStreamNonBlocking, hi));
        if (v >= 4) {
            CK(hipExtStreamCreateWithCUMask(&f, (uint32_t)mask.size(), mask.data()));
            CK(hipExtStreamCreateWithCUMask(&t, (uint32_t)mask.size(), mask.data()));
        } else {
            CK(hipStreamCreateWithFlags(&f, hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
        }
        std::vector<hipEvent_t> evf(L), evc(L);
        for (int i = 0; i < L; i++) {
            CK(hipEventCreateWithFlags(&evf[i], hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&evc[i], hipEventDisableTiming));
        }
        CK(hipMemset(st, 0xff, 8 * L));
        CK(hipMemset(en, 0, 8 * L));
        CK(hipDeviceSynchronize());
        const size_t nw = v == 5 ? nw_big : 0;
        for (int i = 0; i < L; i++) {
            if (v >= 2) {
                if (v >= 3)
                    hipExtLaunchKernelGGL(k_short, dim3(1), dim3(64), 0u, f, nullptr, evf[i], 0u, aux);
                else {
                    k_short<<<1, 64, 0, f>>>(aux);
                    CK(hipEventRecord(evf[i], f));
                }
                CK(hipStreamWaitEvent(c, evf[i], 0));
            }
            hipExtLaunchKernelGGL(k_spin, dim3(grid), dim3(block), (uint32_t)lds, c, nullptr, v >= 3 ? evc[i] : nullptr,
                                  0u, (uint64_t)20000, st, en, i, out, nw);   // 200 us
            if (v >= 3) {
                CK(hipStreamWaitEvent(t, evc[i], 0));
                k_short<<<1, 64, 0, t>>>(aux + 64);
            }
        }
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> hs(L), he(L);
        CK(hipMemcpy(hs.data(), st, 8 * L, hipMemcpyDeviceToHost));
        CK(hipMemcpy(he.data(), en, 8 * L, hipMemcpyDeviceToHost));
        std::vector<double> gap;
        for (int i = 2; i + 1 < L; i++) gap.push_back((double)(hs[i + 1] - he[i]) * 0.01);
        std::sort(gap.begin(), gap.end());
        printf("%-7s gap us: min %.2f median %.2f max %.2f   (launch %.1f us)\n", names[v], gap.front(),
               gap[gap.size() / 2], gap.back(), (double)(he[3] - hs[3]) * 0.01);
        for (int i = 0; i < L; i++) {
            CK(hipEventDestroy(evf[i]));
            CK(hipEventDestroy(evc[i]));
        }
        CK(hipStreamDestroy(c));
        CK(hipStreamDestroy(f));
        CK(hipStreamDestroy(t));
    }
    return 0;
}
