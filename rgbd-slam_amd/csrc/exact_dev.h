// exact_dev.h -- IEEE-exact short sequences for a double sqrt / division on operands whose range is known:
// the sequences the compiler emits on gfx950 minus the range scaling and special-case steps that are identities
// there (v_div_scale / v_div_fmas / v_div_fixup with no scaling and a finite quotient; the sqrt's 2^-767
// pre-scale), so every result has the bits of the IEEE operation (pinned by rgbd_debug_rotation_ops +
// test_rotation_sqrt_div_sequences_are_ieee over 1M operands).  Used by the EPnP Jacobi (pnp.hip) and the
// 3 x 3 SVD (svd3_dev.h).
#pragma once
#include <hip/hip_runtime.h>

namespace rgbd {

// 4-5 fewer dependent steps per sqrt, 2 per division than the general sequences.
// sqrt(x) for finite x >= 1
__device__ __forceinline__ double sqrt_ge1(double x)
{
    const double r = __builtin_amdgcn_rsq(x);
    double g = x * r, h = r * 0.5;
    const double e = fma(-h, g, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
}
// n / d without v_div_scale's range scaling or v_div_fixup: the IEEE quotient for |d| in [1, 2^1000) with n / d
// normal and |n| >= 2^-969, or d == 1 (below ~2^-969 the residual fma(-d, q, n) is subnormal and the quotient is
// exact only when d == 1 -- the case of svd3's u / sqrt(1 + u^2) for tiny u, where sqrt(1 + u^2) rounds to 1)
__device__ __forceinline__ double div_plain(double n, double d)
{
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    const double q = n * r;
    return fma(fma(-d, q, n), r, q);
}

}  // namespace rgbd
