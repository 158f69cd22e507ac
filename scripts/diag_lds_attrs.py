"""Print the device's per-workgroup LDS attributes as HIP reports them
(hipDeviceAttributeMaxSharedMemoryPerBlock = 74, ...SharedMemPerBlockOptin =
75 in ROCm 7.2's hip_runtime_api.h): the version probe sizes its LDS tables
by the larger of the two (bloom_kernels.hip device_lds_max)."""
import ctypes

h = ctypes.CDLL("libamdhip64.so")
for name, attr in (("MaxSharedMemoryPerBlock", 74), ("SharedMemPerBlockOptin", 75)):
    v = ctypes.c_int(0)
    rc = h.hipDeviceGetAttribute(ctypes.byref(v), attr, 0)
    print(name, rc, v.value)
