// Bit-equality probe of two fp16 splits of x * 2^8 (cv_row.hip's left operand), built with cv_row.hip's flags
// (-fno-honor-nans -mno-amdgpu-ieee): (a) per value, hi = (f16)xs, lo = (f16)(xs - (float)hi); (b) pairs, hi by
// one packed convert, lo by v_fma_mix{lo,hi}_f16.  Counts the values whose hi or lo bits differ.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__global__ void split_probe_kernel(const float *__restrict__ x, int64_t n, unsigned *__restrict__ nbad,
                                   uint32_t *__restrict__ first)
{
    const int64_t i = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (i + 1 >= n) return;
    const float scl = 256.0f;
    const float x0 = x[i] * scl, x1 = x[i + 1] * scl;
    const _Float16 a0 = (_Float16)x0, a1 = (_Float16)x1;
    const _Float16 b0 = (_Float16)(x0 - (float)a0), b1 = (_Float16)(x1 - (float)a1);
    const h2 hh = {(_Float16)x0, (_Float16)x1};
    const uint32_t hv = __builtin_bit_cast(uint32_t, hh);
    uint32_t lv;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lv) : "v"(x0), "v"(hv));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lv) : "v"(x1), "v"(hv));
    const h2 ha = {a0, a1}, la = {b0, b1};
    const uint32_t hva = __builtin_bit_cast(uint32_t, ha), lva = __builtin_bit_cast(uint32_t, la);
    if (hva != hv || lva != lv) {
        if (atomicAdd(nbad, 1u) == 0u) {
            first[0] = __float_as_uint(x[i]); first[1] = __float_as_uint(x[i + 1]);
            first[2] = hva; first[3] = hv; first[4] = lva; first[5] = lv;
        }
    }
}

extern "C" int split_probe(const float *x, int64_t n, unsigned *nbad, uint32_t *first, void *stream)
{
    const int64_t pairs = n / 2;
    split_probe_kernel<<<(unsigned)((pairs + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, n, nbad, first);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
