"""Write tools/_var/tower_h16_phase.h: the PRODUCT tower_h16.h with per-phase s_memtime stamps injected (the
round-6 phase probe of tools/variants/tower_h16_diag.h, H16_DIAG & 16384, applied to the current product code so
the probe never drifts from it).  Every wave's lane 0 writes 4 floats to out[32 blockIdx.x + 4 wave ..] at the end:
MFMA waves (c-block loop, epilogue, barrier), stagers (work, barrier).  Timing-only: wrong outputs in tile-0 rows.
usage: python tools/variants/make_phase_header.py && bash tools/build_file_variant.sh tower.hip phase \\
         -DSDE_H16_HEADER='"'$PWD/tools/_var/tower_h16_phase.h'"'   then python tools/tower_phase.py tools/_var/libsde_phase.so"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "scenedepthestimation_amd", "csrc", "tower_h16.h")).read()


def rep(s, old, new):
    assert old in s, old[:70]
    return s.replace(old, new, 1)


helpers = '''__device__ float *h16_probe_out;
__device__ __forceinline__ uint64_t h16_stamp()
{
    const uint64_t t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    return t;
}
__device__ __forceinline__ void h16_stamp_out(float *out, int wave, int lane, const uint64_t (&ph)[4])
{
    if (lane == 0)
        for (int k = 0; k < 4; k++) out[32 * blockIdx.x + 4 * wave + k] = (float)ph[k];
}

'''
s = rep(src, "namespace sde {\n", "namespace sde {\n" + helpers)
s = rep(s, '''#pragma unroll 1
    for (int i = 0; i < nsteps; i++) {
        if (2 * i + 2 < nh) store(ra, 2 * i + 2);
        if (2 * i + 4 < nh) load(ra, 2 * i + 4);
        if (2 * i + 3 < nh) store(rb, 2 * i + 3);
        if (2 * i + 5 < nh) load(rb, 2 * i + 5);
        __syncthreads();
    }
}''', '''    uint64_t ph[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (int i = 0; i < nsteps; i++) {
        const uint64_t t0 = h16_stamp();
        if (2 * i + 2 < nh) store(ra, 2 * i + 2);
        if (2 * i + 4 < nh) load(ra, 2 * i + 4);
        if (2 * i + 3 < nh) store(rb, 2 * i + 3);
        if (2 * i + 5 < nh) load(rb, 2 * i + 5);
        const uint64_t t1 = h16_stamp();
        __syncthreads();
        const uint64_t t2 = h16_stamp();
        ph[0] += t1 - t0;
        ph[1] += t2 - t1;
    }
    h16_stamp_out(h16_probe_out, (st >> 6) + 4, st & 63, ph);
}''')
s = rep(s, '''    if (wave >= 4) {
        if (FIRST) h16_conv1_stager_loop''', '''    h16_probe_out = out;
    if (wave >= 4) {
        if (FIRST) h16_conv1_stager_loop''')
s = rep(s, '''        auto cstep = [&](int cb) {
''', '''        auto cstep = [&](int cb) {
            const uint64_t ta = h16_stamp();
''')
s = rep(s, '''            if (cb == H16_NCB - 1) {
                if (img != sc_img) {''', '''            const uint64_t tb = h16_stamp();
            if (cb == H16_NCB - 1) {
                if (img != sc_img) {''')
s = rep(s, '''            __syncthreads();
            cur ^= 1;
        };''', '''            const uint64_t tc = h16_stamp();
            __syncthreads();
            const uint64_t td = h16_stamp();
            pht[0] += tb - ta;
            pht[1] += tc - tb;
            pht[2] += td - tc;
            cur ^= 1;
        };''')
s = rep(s, '''    int sc_img = -1;
    float sc_u = 1.0f, sc_o = 1.0f;''', '''    uint64_t pht[4] = {0, 0, 0, 0};
    int sc_img = -1;
    float sc_u = 1.0f, sc_o = 1.0f;''')
s = rep(s, '''    if (!LAST) xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
}''', '''    if (!LAST) xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
    h16_stamp_out(out, g, lane, pht);
}''')
os.makedirs(os.path.join(ROOT, "tools", "_var"), exist_ok=True)
open(os.path.join(ROOT, "tools", "_var", "tower_h16_phase.h"), "w").write(s)
print("wrote tools/_var/tower_h16_phase.h")
# variant: the stagers skip their loads and splits (barriers only) -- how much of the MFMA waves' loop excess is
# the stagers' issue on the shared SIMDs
s2 = rep(s, """        const uint64_t t0 = h16_stamp();
        if (2 * i + 2 < nh) store(ra, 2 * i + 2);
        if (2 * i + 4 < nh) load(ra, 2 * i + 4);
        if (2 * i + 3 < nh) store(rb, 2 * i + 3);
        if (2 * i + 5 < nh) load(rb, 2 * i + 5);""", """        const uint64_t t0 = h16_stamp();""")
open(os.path.join(ROOT, "tools", "_var", "tower_h16_phase_nostage.h"), "w").write(s2)
print("wrote tools/_var/tower_h16_phase_nostage.h")
