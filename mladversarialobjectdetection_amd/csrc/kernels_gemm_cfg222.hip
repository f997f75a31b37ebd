// kernels_gemm_cfg222.hip — k_gemm2 instantiations of the <2, 2, 2> tile (gemm2_kernel.hpp), one
// translation unit per tile so the GEMM variants compile in parallel.
#include "gemm2_kernel.hpp"

namespace phx {
PHX_G2_DEFINE_LAUNCH_CFG
template void g2_launch_cfg<2, 2, 2, 1>(int, int, dim3, hipStream_t, const Gemm2Group<1>&, bool, int, size_t);
template void g2_launch_cfg<2, 2, 2, kMaxSeg>(int, int, dim3, hipStream_t, const Gemm2Group<kMaxSeg>&, bool, int, size_t);
}  // namespace phx
