// omp_env.cpp -- the OpenMP runtime's wait policy for the library's host threads.
//
// hipcc -fopenmp links LLVM's libomp, whose idle workers spin for KMP_BLOCKTIME (200 ms by default)
// after every parallel region.  The LASolver set-up runs its schedule builders on three helper
// threads, each with its own team, beside the main thread's team: up to ~40 spinning workers on the
// job's 16 CPUs, which slowed the set-up itself and the host-driven Newton/CG-STAB loop of the
// backward-Euler steps right after it (2D steady step 33 -> 39-46 ms; OMP_WAIT_POLICY=passive
// restored it and took the first step 1.02 -> 0.90 s).  libomp reads its environment when it
// initialises, at the first OpenMP construct, which in this process is the library's own: a
// blocktime of 1 ms is set here at load unless the caller chose one.
#include <cstdlib>

namespace {
__attribute__((constructor)) void mmx_omp_blocktime() {
  if (!std::getenv("KMP_BLOCKTIME") && !std::getenv("OMP_WAIT_POLICY")) setenv("KMP_BLOCKTIME", "1", 0);
}
}  // namespace
