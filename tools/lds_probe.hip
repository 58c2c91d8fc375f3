// LDS probe: workgroups of 256 threads, each declaring NB bytes of dynamic LDS, fill their
// whole allocation with a (block, index) pattern, then re-read it many times (b32 / b64 / b128
// accesses) and count mismatches.  With NB > 64 KiB two workgroups share a CU and the second
// one's allocation lies above 128 KiB.  Prints the mismatch count per access width and the
// first bad (block, index, lane) triples.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_probe.hip -o tools/_var/lds_probe
//   tools/_var/lds_probe [NB] [GRID]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(256) void probe(unsigned *err, unsigned *first, int nbytes, int width)
{
    extern __shared__ __attribute__((aligned(16))) unsigned sm[];
    const int n = nbytes / 4;
    const unsigned tag = (unsigned)blockIdx.x << 20;
    for (int i = threadIdx.x; i < n; i += 256) sm[i] = tag + i;
    __syncthreads();
    unsigned bad = 0;
    for (int rep = 0; rep < 64; rep++) {
        if (width == 4) {
            for (int i = threadIdx.x; i < n; i += 256)
                if (sm[i] != tag + i) { bad++; if (atomicCAS(first, 0u, 1u) == 0u) { first[1] = blockIdx.x; first[2] = i; first[3] = threadIdx.x; first[4] = sm[i]; } }
        } else if (width == 8) {
            const uint2 *s2 = reinterpret_cast<const uint2 *>(sm);
            for (int i = threadIdx.x; i < n / 2; i += 256) {
                const uint2 v = s2[i];
                if (v.x != tag + 2 * i || v.y != tag + 2 * i + 1) { bad++; if (atomicCAS(first, 0u, 1u) == 0u) { first[1] = blockIdx.x; first[2] = 2 * i; first[3] = threadIdx.x; first[4] = v.x; } }
            }
        } else {
            const uint4 *s4 = reinterpret_cast<const uint4 *>(sm);
            for (int i = threadIdx.x; i < n / 4; i += 256) {
                const uint4 v = s4[i];
                if (v.x != tag + 4 * i || v.y != tag + 4 * i + 1 || v.z != tag + 4 * i + 2 || v.w != tag + 4 * i + 3) {
                    bad++;
                    if (atomicCAS(first, 0u, 1u) == 0u) { first[1] = blockIdx.x; first[2] = 4 * i; first[3] = threadIdx.x; first[4] = v.x; }
                }
            }
        }
    }
    if (bad) atomicAdd(&err[blockIdx.x], bad);
}

int main(int argc, char **argv)
{
    const int nb = argc > 1 ? atoi(argv[1]) : 78592;
    const int grid = argc > 2 ? atoi(argv[2]) : 512;
    hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, nb);
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, probe, 256, nb);
    unsigned *err, *first;
    hipMalloc(&err, grid * 4);
    hipMalloc(&first, 64);
    for (int width : {4, 8, 16}) {
        hipMemset(err, 0, grid * 4);
        hipMemset(first, 0, 64);
        probe<<<grid, 256, nb>>>(err, first, nb, width);
        hipError_t e = hipDeviceSynchronize();
        std::vector<unsigned> h(grid), f(5);
        hipMemcpy(h.data(), err, grid * 4, hipMemcpyDeviceToHost);
        hipMemcpy(f.data(), first, 20, hipMemcpyDeviceToHost);
        unsigned long long tot = 0;
        int nbad = 0;
        for (int b = 0; b < grid; b++) { tot += h[b]; nbad += h[b] != 0; }
        printf("LDS %d B/workgroup, grid %d, occupancy %d/CU, %d-B reads: %s, mismatches %llu in %d workgroups",
               nb, grid, occ, width, hipGetErrorString(e), tot, nbad);
        if (tot) printf("; first: block %u word %u (byte %u) thread %u read 0x%08x", f[1], f[2], f[2] * 4, f[3], f[4]);
        printf("\n");
    }
    return 0;
}
