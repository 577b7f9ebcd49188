// runtime.hip — device selection and status reporting for the C ABI
// (include/x265_amd.h).  x265 has no error channel inside its primitives
// (primitives.h typedefs); failures surface as non-zero status codes here and
// are mapped by the caller onto x265_encoder_open() == NULL /
// x265_encoder_encode() < 0 (x265.h:1351-1359).
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../../include/x265_amd.h"

extern "C" int x265amd_abi_version(void)
{
    return X265AMD_ABI_VERSION;
}

extern "C" const char* x265amd_target(void)
{
    return "gfx950";
}

extern "C" int x265amd_device_count(int* count)
{
    if (!count) return X265AMD_EINVAL;
    *count = 0;
    const hipError_t e = hipGetDeviceCount(count);
    if (e == hipErrorNoDevice)
    {
        *count = 0;
        return 0;
    }
    return (int)e;
}

extern "C" int x265amd_set_device(int device)
{
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess) return (int)e;
    if (device < 0 || device >= count) return X265AMD_ENODEV;
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return (int)e;
    // code objects are built for gfx950 only: refuse any other target loudly
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return X265AMD_ENODEV;
    return (int)hipSetDevice(device);
}

extern "C" const char* x265amd_strerror(int status)
{
    switch (status)
    {
    case X265AMD_OK: return "success";
    case X265AMD_EINVAL: return "x265amd: unsupported primitive, block shape or bit depth";
    case X265AMD_ENODEV: return "x265amd: no gfx950 (MI355X) device";
    case X265AMD_ENOMEM: return "x265amd: device or pinned staging allocation failed";
    default: return hipGetErrorString((hipError_t)status);
    }
}

/* sizeof of a descriptor type of include/x265_amd.h by name (0 if unknown): lets a binding written in
 * another language (the ctypes structures of src/x265_amd/native.py) check its layouts against the
 * library's (tests/test_capi.py) */
extern "C" int x265amd_sizeof(const char* type)
{
    if (!type) return 0;
#define T(name) if (!strcmp(type, #name)) return (int)sizeof(name);
    T(x265amd_cmp_batch) T(x265amd_interp_batch) T(x265amd_block_batch) T(x265amd_tu_batch)
    T(x265amd_lowres_batch) T(x265amd_lowres_intra_batch) T(x265amd_lowres_pcost_batch) T(x265amd_lowres_bcost_batch)
    T(x265amd_la_config) T(x265amd_la_pjob) T(x265amd_la_bjob) T(x265amd_sched_config) T(x265amd_sched_frame)
    T(x265amd_transfer) T(x265amd_propagate_batch) T(x265amd_weights_batch) T(x265amd_me_batch) T(x265amd_mes_config)
    T(x265amd_mes_job) T(x265amd_mes_counters) T(x265amd_sao_param) T(x265amd_sao_frame) T(x265amd_sao_stats_frame)
    T(x265amd_deblock_unit) T(x265amd_deblock_frame) T(x265amd_border_plane)
#undef T
    return 0;
}
