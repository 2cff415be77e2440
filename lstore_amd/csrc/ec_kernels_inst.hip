// ec_kernels_inst.hip -- explicit instantiation of the kernels for R = LSEC_R output rows.
// The Makefile compiles this file once per R (1..8) with -DLSEC_R=<R>.
#define LSEC_INSTANTIATING 1
#include "ec_kernels_impl.h"

#ifndef LSEC_R
#error "compile with -DLSEC_R=<rows>"
#endif

namespace lsec {
template hipError_t dispatch_bytewise<LSEC_R>(const ApplyArgs &, hipStream_t, int, int);
template hipError_t dispatch_bitsliced<LSEC_R>(const ApplyArgs &, hipStream_t, int, int);
template hipError_t dispatch_bitmatrix<LSEC_R>(const ApplyArgs &, hipStream_t, int);
template hipError_t dispatch_bytewise_magic<LSEC_R>(const ApplyArgs &, hipStream_t, int);
template hipError_t dispatch_wordwise<LSEC_R>(const ApplyArgs &, hipStream_t, int);
template hipError_t dispatch_gfw_bitsliced<LSEC_R>(const ApplyArgs &, hipStream_t, int);
template hipError_t dispatch_gfw_transposed<LSEC_R>(const ApplyArgs &, hipStream_t, int);
}  // namespace lsec
