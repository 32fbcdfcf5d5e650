// Issue-rate probe (gfx950): wave-instructions per cycle per CU for a stream of
// independent SALU adds vs VALU adds vs both interleaved, at 1..8 waves per SIMD.
// Tells whether the scalar ALU is a per-SIMD or a per-CU resource (DESIGN.md
// section 4 "What bounds it").  usage: ./issue_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int KIND>
__global__ void __launch_bounds__(256) k_probe(unsigned* out, unsigned long long* cyc, int iters)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    unsigned sa = blockIdx.x, sb = sa + 1, sc = sa + 2, sd = sa + 3;
    for (int i = 0; i < iters; i++) {
        if (KIND == 0 || KIND == 2)
            asm volatile("s_add_u32 %0, %0, 1\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %2, %2, 1\n\ts_add_u32 %3, %3, 1\n\t"
                         "s_add_u32 %0, %0, 1\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %2, %2, 1\n\ts_add_u32 %3, %3, 1"
                         : "+s"(sa), "+s"(sb), "+s"(sc), "+s"(sd)
                         :
                         : "scc");
        if (KIND == 1 || KIND == 2)
            asm volatile("v_add_u32 %0, %0, 1\n\tv_add_u32 %1, %1, 1\n\tv_add_u32 %2, %2, 1\n\tv_add_u32 %3, %3, 1\n\t"
                         "v_add_u32 %0, %0, 1\n\tv_add_u32 %1, %1, 1\n\tv_add_u32 %2, %2, 1\n\tv_add_u32 %3, %3, 1"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    }
    out[blockIdx.x * 256 + threadIdx.x] = a + b + c + d + sa + sb + sc + sd;
    __syncthreads();
    if (threadIdx.x == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;   // shader cycles
}

int main()
{
    setvbuf(stdout, nullptr, _IONBF, 0);
    int dev = 0, cus = 0, clk = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);   // kHz
    unsigned* out;
    unsigned long long* cyc;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    hipMalloc(&cyc, (size_t)cus * 8 * 8);
    unsigned long long* hc = (unsigned long long*)malloc((size_t)cus * 8 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    const char* names[3] = {"salu", "valu", "salu+valu"};
    for (int kind = 0; kind < 3; kind++)
        for (int bpc = 1; bpc <= 8; bpc *= 2) {   // blocks of 4 waves per CU: waves/SIMD = bpc
            const int grid = cus * bpc;
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (kind == 0) hipLaunchKernelGGL(k_probe<0>, dim3(grid), dim3(256), 0, 0, out, cyc, iters);
                if (kind == 1) hipLaunchKernelGGL(k_probe<1>, dim3(grid), dim3(256), 0, 0, out, cyc, iters);
                if (kind == 2) hipLaunchKernelGGL(k_probe<2>, dim3(grid), dim3(256), 0, 0, out, cyc, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep == 1) {
                    hipMemcpy(hc, cyc, (size_t)grid * 8, hipMemcpyDeviceToHost);
                    unsigned long long mx = 0;
                    for (int b = 0; b < grid; b++) mx = hc[b] > mx ? hc[b] : mx;
                    const double insts = (double)iters * 8 * (kind == 2 ? 2 : 1) * grid * 4;   // wave-instructions
                    printf("%-10s waves/SIMD %d  %.3f ms  %.3f wave-instr/shader-cycle/CU  (block span %llu cycles, "
                           "effective clock %.0f MHz)\n", names[kind], bpc, ms, insts / cus / (double)mx, mx,
                           (double)mx / (ms * 1e3));
                }
            }
        }
    hipFree(out);
    return 0;
}
