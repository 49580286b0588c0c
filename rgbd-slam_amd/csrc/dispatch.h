// dispatch.h -- the one way a launcher in this library puts a kernel on a stream (included by the .hip files).
//
// Every dispatch is checked on the host before it is queued, and its own status is returned:
//   * an empty grid (a dimension of 0) is "no work": nothing is queued and hipSuccess returned;
//   * grid.y / grid.z <= 65535, block <= 1024 threads, and grid x block work-items per dimension within the
//     32-bit grid_size fields of the AQL dispatch packet;
//   * dynamic + static LDS within the 160 KiB one gfx950 workgroup may hold; dynamic LDS above 64 KiB is
//     opted into per kernel (hipFuncSetAttribute, once per kernel and size) and that call's status is checked;
//   * the launch's status (hipGetLastError right after the launch: HIP sets it per API call).
// The host code turns any failure into RGBD_ERR_HIP (check_hip) instead of queueing a malformed dispatch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <utility>

namespace rgbd {

constexpr size_t kLdsPerWorkgroup = 160 * 1024;   // gfx950: the whole CU's LDS may go to one workgroup
constexpr size_t kLdsDefaultLimit = 64 * 1024;    // dynamic LDS above this needs the per-kernel opt-in

// Per (device, kernel), looked up / set once: its static LDS (hipFuncGetAttributes) and the dynamic LDS it is
// opted into (hipFuncSetAttribute applies to the current device, so the opt-in is kept per device and called
// again only when a launch on that device needs more than its last opt-in)
struct KernelLds {
    int dev;
    const void* k;
    size_t fixed, optin;
};
inline hipError_t kernel_lds(const void* k, size_t dyn, size_t* fixed)
{
    static std::mutex mu;
    static KernelLds tab[256];
    static int n = 0;
    int dev = 0;
    const hipError_t de = hipGetDevice(&dev);
    if (de != hipSuccess) return de;
    std::lock_guard<std::mutex> lock(mu);
    KernelLds* e = nullptr;
    for (int i = 0; i < n; i++)
        if (tab[i].k == k && tab[i].dev == dev) e = &tab[i];
    KernelLds tmp{dev, k, 0, kLdsDefaultLimit};
    if (!e) {
        hipFuncAttributes a{};
        const hipError_t r = hipFuncGetAttributes(&a, k);
        if (r != hipSuccess) return r;
        tmp.fixed = a.sharedSizeBytes;
        e = n < 256 ? &tab[n++] : &tmp;
        *e = tmp;
    }
    *fixed = e->fixed;
    if (dyn + e->fixed > kLdsPerWorkgroup) return hipErrorInvalidValue;
    if (dyn > e->optin) {
        const hipError_t r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
        if (r != hipSuccess) return r;
        e->optin = dyn;
    }
    return hipSuccess;
}

template <typename... P, typename... A>
hipError_t dispatch(void (*k)(P...), dim3 grid, dim3 block, size_t lds, hipStream_t st, A&&... args)
{
    if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;
    const uint64_t thr = (uint64_t)block.x * block.y * block.z;
    if (thr == 0 || thr > 1024 || grid.y > 65535 || grid.z > 65535 || (uint64_t)grid.x * block.x > 0xFFFFFFFFull ||
        (uint64_t)grid.y * block.y > 0xFFFFFFFFull || (uint64_t)grid.z * block.z > 0xFFFFFFFFull)
        return hipErrorInvalidConfiguration;
    if (lds > 0) {
        size_t fixed = 0;
        const hipError_t e = kernel_lds(reinterpret_cast<const void*>(k), lds, &fixed);
        if (e != hipSuccess) return e;
    }
    (void)hipGetLastError();   // a stale status of an earlier call must not be read as this launch's
    k<<<grid, block, lds, st>>>(std::forward<A>(args)...);
    return hipGetLastError();
}

}  // namespace rgbd
