// FETCH_SIZE calibration reads (scripts/calib/fetch_calib.py): every byte of a device buffer read
// exactly once, with the per-lane widths the likelihood kernel issues (8 B: global_load_dwordx2,
// 16 B: global_load_dwordx4), one sum per lane written out. The rocprofv3 FETCH_SIZE of each
// dispatch divided by the bytes read is the counter's factor for that load shape on gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int W>  // doubles per lane and load: 1 (8 B) or 2 (16 B)
__global__ __launch_bounds__(256) void calib_read(const double* __restrict__ src, double* __restrict__ dst, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x, nt = (int64_t)gridDim.x * 256;
  double s = 0.0;
  if (W == 1) {
    for (int64_t i = t; i < n; i += nt) s += src[i];
  } else {
    const double2* s2 = reinterpret_cast<const double2*>(src);
    for (int64_t i = t; i < n / 2; i += nt) {
      const double2 v = s2[i];
      s += v.x + v.y;
    }
  }
  dst[t] = s;
}

extern "C" int calib_launch(const double* src, double* dst, int64_t n, int width, int blocks, void* stream) {
  if (width == 1)
    hipLaunchKernelGGL(calib_read<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, dst, n);
  else
    hipLaunchKernelGGL(calib_read<2>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, dst, n);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
