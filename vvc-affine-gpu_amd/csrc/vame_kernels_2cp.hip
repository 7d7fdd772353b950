// The 2-CP-only (MODE 1) product kernels, in a translation unit of their own:
// the Makefile builds it without SimplifyCFG's hoisting and sinking of common
// code (the flags that suit these two-body kernels); the engine
// (vame_engine.hip) declares them.  Instrumentation builds instantiate them in
// the engine's unit instead (vame_kernel.h, VAME_SPLIT_TU).
#include "vame_kernel.h"

#if VAME_SPLIT_TU
namespace vame {
VAME_2CP_KERNELS()
}
#endif
