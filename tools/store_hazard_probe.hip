// store_hazard_probe.hip -- does a VALU write to the first data VGPR of a buffer_store_dwordx4 issued right
// after the store corrupt the stored value on gfx950 ("store-data overwrite")?
//
// One 512-thread workgroup per CU: waves 0-3 (one per SIMD) run a dense v_mfma_f32_32x32x16_f16 loop
// (or idle, MFMA = 0), waves 4-7 share those SIMDs and, N times, write a known float4 with
// buffer_store_dwordx4 (register soffset, the case LLVM's hazard recognizer treats as safe) and overwrite
// the first data register with a poison value GAP wait states later -- all in one asm block, so the
// instruction order is exactly that.  The host counts stored float4s whose first dword is the poison.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/_var/store_hazard_probe tools/store_hazard_probe.hip
//   tools/_var/store_hazard_probe     (prints one line per (MFMA on/off, gap) case)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int N = 2048;             // stores per store-wave
constexpr unsigned POISON = 0x7fbadbadu;

template <int GAP, bool MFMA>
__global__ __launch_bounds__(512) void probe(unsigned *out, int iters)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave < 4) {
        if (!MFMA) return;
        f16x8 a, b;
        for (int i = 0; i < 8; i++) {
            a[i] = (_Float16)(0.001f * (lane + i));
            b[i] = (_Float16)(0.002f * (lane - i));
        }
        floatx16 c = {0};
        for (int i = 0; i < iters; i++) {
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c, 0, 0, 0);
        }
        if (c[0] == 12345.f) out[0] = 1;   // keep the loop
        return;
    }
    const int sw = wave - 4;
    unsigned *base = out + ((size_t)(blockIdx.x * 4 + sw) * N) * 256;   // N float4 x 64 lanes per wave
    const uintptr_t b = (uintptr_t)base;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 rs;   // raw buffer descriptor: base, 1 GiB of records
    rs.x = __builtin_amdgcn_readfirstlane((unsigned)b);
    rs.y = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32)) & 0xffffu;
    rs.z = 0x40000000u;
    rs.w = 0x00020000u;
    const unsigned voff = 16u * lane;
    for (int i = 0; i < N; i++) {
        const unsigned so = (unsigned)i * 1024u;   // this store's row: a register soffset
        const unsigned v0 = (unsigned)(i * 64 + lane) * 4u;
        if (GAP == 0)
            asm volatile("v_mov_b32 v40, %0\n\tv_add_u32 v41, 1, %0\n\tv_add_u32 v42, 2, %0\n\tv_add_u32 v43, 3, %0\n\t"
                         "buffer_store_dwordx4 v[40:43], %1, %2, %3 offen\n\t"
                         "v_mov_b32 v40, %4\n\t"
                         "s_nop 7\n\ts_nop 7"
                         :: "v"(v0), "v"(voff), "s"(rs), "s"(so), "v"(POISON) : "v40", "v41", "v42", "v43", "memory");
        else if (GAP == 1)
            asm volatile("v_mov_b32 v40, %0\n\tv_add_u32 v41, 1, %0\n\tv_add_u32 v42, 2, %0\n\tv_add_u32 v43, 3, %0\n\t"
                         "buffer_store_dwordx4 v[40:43], %1, %2, %3 offen\n\t"
                         "s_nop 0\n\t"
                         "v_mov_b32 v40, %4\n\t"
                         "s_nop 7\n\ts_nop 7"
                         :: "v"(v0), "v"(voff), "s"(rs), "s"(so), "v"(POISON) : "v40", "v41", "v42", "v43", "memory");
        else
            asm volatile("v_mov_b32 v40, %0\n\tv_add_u32 v41, 1, %0\n\tv_add_u32 v42, 2, %0\n\tv_add_u32 v43, 3, %0\n\t"
                         "buffer_store_dwordx4 v[40:43], %1, %2, %3 offen\n\t"
                         "s_nop 4\n\t"
                         "v_mov_b32 v40, %4\n\t"
                         "s_nop 7\n\ts_nop 7"
                         :: "v"(v0), "v"(voff), "s"(rs), "s"(so), "v"(POISON) : "v40", "v41", "v42", "v43", "memory");
    }
}

template <int GAP, bool MFMA>
static void run(unsigned *d, std::vector<unsigned> &h, int ncu, size_t words)
{
    hipMemset(d, 0, words * 4);
    probe<GAP, MFMA><<<ncu, 512>>>(d, 40000);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("launch failed\n");
        exit(1);
    }
    hipMemcpy(h.data(), d, words * 4, hipMemcpyDeviceToHost);
    size_t bad = 0, poison = 0, checked = 0;
    for (int blk = 0; blk < ncu; blk++)
        for (int sw = 0; sw < 4; sw++)
            for (int i = 0; i < N; i++)
                for (int l = 0; l < 64; l++) {
                    const size_t w = (((size_t)(blk * 4 + sw) * N + i) * 64 + l) * 4;
                    const unsigned v0 = (unsigned)(i * 64 + l) * 4u;
                    checked++;
                    if (h[w] == POISON) poison++;
                    if (h[w] != v0 || h[w + 1] != v0 + 1 || h[w + 2] != v0 + 2 || h[w + 3] != v0 + 3) bad++;
                }
    printf("MFMA waves %-3s  gap %s: %zu of %zu float4 wrong (%zu with the poison in the first dword)\n",
           MFMA ? "on" : "off", GAP == 0 ? "0 (next instruction)" : GAP == 1 ? "1 (s_nop 0)" : "5 (s_nop 4)", bad,
           checked, poison);
}

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t words = (size_t)ncu * 4 * N * 256;
    unsigned *d = nullptr;
    if (hipMalloc(&d, words * 4) != hipSuccess) return 1;
    std::vector<unsigned> h(words);
    for (int rep = 0; rep < 2; rep++) {
        run<0, false>(d, h, ncu, words);
        run<0, true>(d, h, ncu, words);
        run<1, true>(d, h, ncu, words);
        run<2, true>(d, h, ncu, words);
    }
    hipFree(d);
    return 0;
}
