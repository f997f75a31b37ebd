// kernels_gemm_cfg413.hip — k_gemm2 instantiations of the <4, 1, 3> tile (gemm2_kernel.hpp), one
// translation unit per tile so the GEMM variants compile in parallel.
#include "gemm2_kernel.hpp"

namespace phx {
PHX_G2_DEFINE_LAUNCH_CFG
template void g2_launch_cfg<4, 1, 3, 1>(int, int, dim3, hipStream_t, const Gemm2Group<1>&, bool, int, size_t);
template void g2_launch_cfg<4, 1, 3, kMaxSeg>(int, int, dim3, hipStream_t, const Gemm2Group<kMaxSeg>&, bool, int, size_t);
}  // namespace phx
