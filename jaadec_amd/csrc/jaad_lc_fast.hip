// The +-1 LSB instantiations of lc_decode_kernel (kernel modes 4 and 6, jaad_stream_cfg.precision =
// JAAD_PRECISION_LSB1): jaad_lc.hip compiled a second time with JAAD_LC_FAST_TU, so that these
// kernels get their own compiler flags (jaadec_amd/build.py GPU_FILE_FLAGS: the iterative-ILP machine
// scheduler).  jaad_lc.hip's launch_lc calls launch_lc_fast for them; the other modes and every
// other entry point are compiled only there.
#define JAAD_LC_FAST_TU
#include "jaad_lc.hip"
