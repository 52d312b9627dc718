// layout.h -- the one place for every compile-time switch that changes the layout of a buffer
// written by host code and read by a kernel (or the other way round).  Host and kernel
// translation units include this header; each kernel object exports the layout word it was
// compiled with (mmx_layout_admm / _sparse / _chain, extern "C"), and the host compares them with
// its own before any HIP call (check_kernel_layout, host/layout_check.cpp): a library whose host and
// kernel objects were built with different switches fails at create with MMADMM_ERR_INVALID
// instead of computing on a misread buffer (round 5's z/u mismatch reached the GPU that way).
#pragma once

// 2D z / u: 1 = interleaved per vertex slot (admm_kernels.hip zu_*), 0 = two arrays (kept:
// interleaved measured slower, C3 x-update 0.063 -> 0.068 ms, prox 0.325 -> 0.330 ms; profiles/r05/ab/)
#ifndef MMX_ZU_INTER
#define MMX_ZU_INTER 0
#endif
// SpMV row blocks built on the host (sparse.cpp) for the kernel's LDS tile (sparse_kernels.hip)
#ifndef MMX_SPMV_TILE
#define MMX_SPMV_TILE 2048
#endif
#ifndef MMX_SPMV_BLOCK
#define MMX_SPMV_BLOCK 256
#endif
// chain-sweep stage images (chain_sweep.hip, host/sparse.cpp upload_chain): entries lane-interleaved
// for 16-byte LDS reads (MMX_CHAIN_VEC), entry codes 16-bit (MMX_CHAIN_CODE16; 32-bit otherwise,
// except the 48-entry stages, always 16-bit)
// 3D Bkinv wave blocks with each lane's entries in pairs: entry ij of simplex s at
// ((s / 64) K^2 + (ij & ~1)) 64 + 2 (s % 64) + (ij & 1), so a lane's row is 16-byte accesses
#ifndef MMX_B3_PAIRS
#define MMX_B3_PAIRS 1
#endif
#ifndef MMX_CHAIN_VEC
#define MMX_CHAIN_VEC 1
#endif
#ifndef MMX_CHAIN_CODE16
#define MMX_CHAIN_CODE16 1
#endif

namespace mmx {
// the partial-sum record of a workgroup (admm_kernels.h) and the Bkinv wave block of bidx<D>
// (admm_kernels.hip; the engine's host mirror bIndex) are part of the word too
constexpr unsigned kLayoutPartials = 6;
constexpr unsigned kLayoutBkinvBlock = 64;
constexpr unsigned kLayoutWord = 0x4d000000u | ((unsigned)(MMX_ZU_INTER != 0) << 0) |
                                 ((unsigned)(MMX_CHAIN_VEC != 0) << 1) | ((unsigned)(MMX_CHAIN_CODE16 != 0) << 2) |
                                 (((unsigned)MMX_SPMV_TILE / 256u & 0xFu) << 4) |
                                 (((unsigned)MMX_SPMV_BLOCK / 64u & 0xFu) << 8) | ((kLayoutPartials & 0xFu) << 12) |
                                 ((kLayoutBkinvBlock / 64u & 0x3u) << 16) | ((unsigned)(MMX_B3_PAIRS != 0) << 18);
}  // namespace mmx
