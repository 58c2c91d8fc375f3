// Shared helpers for the libsde HIP sources (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <type_traits>

#include "sde.h"

#define SDE_EXPORT extern "C" __attribute__((visibility("default")))

namespace sde {

static inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

static inline int launch_status()
{
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SDE_OK : SDE_ERR_LAUNCH;
}

static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Per-device one-time setup (kernel attributes such as the >64 KB dynamic-LDS opt-in are per
// device): `done` holds one bit per device id; the first caller on a device runs `fn` and
// publishes the bit.  Concurrent first calls may both run `fn`, which is idempotent.  A callback
// returning bool publishes the bit only on success (a failed setup is retried by the next call,
// and every call returns whether the setup holds); a void callback always publishes.
template <typename F>
static inline bool once_per_device(std::atomic<uint64_t> &done, F fn)
{
    constexpr bool checked = std::is_same<decltype(fn()), bool>::value;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        if constexpr (checked) return fn();
        fn();
        return true;
    }
    const uint64_t bit = 1ull << dev;
    if (done.load(std::memory_order_acquire) & bit) return true;
    bool ok = true;
    if constexpr (checked) ok = fn();
    else fn();
    if (ok) done.fetch_or(bit, std::memory_order_acq_rel);
    return ok;
}

// 64-float (256 B) rows in LDS, XOR-swizzled at 16-B granularity: the 16 lanes
// of one ds_read_b128 group that read the same logical chunk of 16 consecutive
// rows land on 16 distinct 16-B slots of the 256-B bank row (conflict-free).
__device__ __forceinline__ int swz_row16(int row, int chunk) { return row * 16 + (chunk ^ (row & 15)); }

// NumPy float32 pairwise sum of elementwise products, 0.0f + pairwise(a*b)
// (numpy loops_utils.h.src pairwise_sum; add.reduce identity 0.0).  Products
// and sums are separately rounded: the library is built with -ffp-contract=off.
__device__ static float pw_prod_rec(const float *a, const float *b, int n)
{
    if (n < 8) {
        float res = 0.0f;
        for (int i = 0; i < n; i++) res += a[i] * b[i];
        return res;
    }
    if (n <= 128) {
        float r[8];
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] = a[j] * b[j];
        int i = 8;
        for (; i < n - (n % 8); i += 8) {
#pragma unroll
            for (int j = 0; j < 8; j++) r[j] += a[i + j] * b[i + j];
        }
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i] * b[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_prod_rec(a, b, n2) + pw_prod_rec(a + n2, b + n2, n - n2);
}

__device__ __forceinline__ float np_neg_dot(const float *a, const float *b, int n)
{
    float s = 0.0f + pw_prod_rec(a, b, n);
    return -s;
}

// First-min merge: b replaces a iff it is strictly smaller, or equal with a lower
// index -- the sequential `v < best` scan's answer for any split of the d range.
__device__ __forceinline__ void argmin_merge(float &ma, int &aa, float mb, int ab)
{
    if (mb < ma || (mb == ma && ab < aa)) {
        ma = mb;
        aa = ab;
    }
}

}  // namespace sde
