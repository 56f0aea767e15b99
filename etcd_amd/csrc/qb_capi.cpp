// qb_capi.cpp — library-level C ABI: version, per-thread error text, devices.
#include <cstdarg>
#include <cstdio>

#include "qb_common.h"

namespace qb {

namespace {
thread_local char t_err[512] = "";
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(t_err, sizeof t_err, fmt, ap);
  va_end(ap);
}

int hip_fail(hipError_t e, const char* what) {
  set_error("%s: %s (%d)", what, hipGetErrorString(e), int(e));
  return QB_EHIP;
}

}  // namespace qb

extern "C" int qb_abi_version(void) { return QB_ABI_VERSION; }

extern "C" const char* qb_last_error(void) { return qb::t_err; }

extern "C" int qb_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky error; "no GPU" is not a failure
    return 0;
  }
  return n;
}

// ------------------------------------------------ memory / stream helpers --

using qb::hip_fail;

extern "C" int qb_set_device(int device) {
  hipError_t e = hipSetDevice(device);
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipSetDevice");
}

extern "C" int qb_malloc(size_t bytes, void** out) {
  if (!out) {
    qb::set_error("qb_malloc: out is NULL");
    return QB_EINVAL;
  }
  *out = nullptr;
  hipError_t e = hipMalloc(out, bytes ? bytes : 1);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    qb::set_error("qb_malloc: out of device memory (%zu bytes)", bytes);
    return QB_ENOMEM;
  }
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipMalloc");
}

extern "C" int qb_free(void* ptr) {
  hipError_t e = hipFree(ptr);
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipFree");
}

extern "C" int qb_memset_async(void* dst, int value, size_t bytes, void* stream) {
  hipError_t e = hipMemsetAsync(dst, value, bytes, qb::as_stream(stream));
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipMemsetAsync");
}

extern "C" int qb_copy_h2d_async(void* dst, const void* src, size_t bytes, void* stream) {
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, qb::as_stream(stream));
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipMemcpyAsync(H2D)");
}

extern "C" int qb_copy_d2h_async(void* dst, const void* src, size_t bytes, void* stream) {
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, qb::as_stream(stream));
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipMemcpyAsync(D2H)");
}

extern "C" int qb_stream_create(void** out) {
  if (!out) {
    qb::set_error("qb_stream_create: out is NULL");
    return QB_EINVAL;
  }
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  *out = s;
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipStreamCreate");
}

extern "C" int qb_stream_destroy(void* stream) {
  hipError_t e = hipStreamDestroy(qb::as_stream(stream));
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipStreamDestroy");
}

extern "C" int qb_stream_sync(void* stream) {
  hipError_t e = hipStreamSynchronize(qb::as_stream(stream));
  return e == hipSuccess ? QB_OK : hip_fail(e, "hipStreamSynchronize");
}
