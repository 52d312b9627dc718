// layout_check.cpp -- host side of layout.h: the layout word of every kernel object must equal the
// word of the host translation unit that creates the objects reading them (engine.cpp, sparse.cpp
// pass their own compile-time kLayoutWord), or nothing is created (MMADMM_ERR_INVALID before any
// HIP call).
#include <cstdio>
#include <string>

#include "../kernels/layout.h"
#include "common.h"

extern "C" unsigned mmx_layout_admm(void);
extern "C" unsigned mmx_layout_sparse(void);
extern "C" unsigned mmx_layout_chain(void);

namespace mmx {

void check_kernel_layout(unsigned hostWord) {
  const struct {
    const char* name;
    unsigned word;
  } objs[] = {{"admm_kernels", mmx_layout_admm()}, {"sparse_kernels", mmx_layout_sparse()},
              {"chain_sweep", mmx_layout_chain()}};
  for (const auto& o : objs)
    if (o.word != hostWord) {
      char buf[256];
      std::snprintf(buf, sizeof buf,
                    "buffer layout mismatch: the %s kernel object was built with layout word 0x%08x, the host "
                    "code with 0x%08x (layout.h switches: MMX_ZU_INTER, MMX_CHAIN_VEC, MMX_CHAIN_CODE16, "
                    "MMX_SPMV_TILE / BLOCK) -- rebuild the library with one set of flags",
                    o.name, o.word, hostWord);
      throw Error(MMADMM_ERR_INVALID, buf);
    }
}

}  // namespace mmx

extern "C" int mmadmm_layout_check(unsigned* host_word) {
  return mmx::guarded([&] {
    if (host_word) *host_word = mmx::kLayoutWord;
    mmx::check_kernel_layout(mmx::kLayoutWord);
  });
}
