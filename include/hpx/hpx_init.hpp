// hpx/hpx_init.hpp -- HPX's explicit start-up shape (hpx::init runs the
// user's hpx_main, hpx::finalize ends it; hpx/hpx_init.hpp in HPX 1.4.0).
// The HIP backend has no AGAS/thread-manager to boot: init checks that the
// library implements the C ABI this header set was written against, then
// calls hpx_main on the calling thread and returns its result.
#pragma once

#include <hpxhip.h>

#include <cstdio>

int hpx_main(int argc, char* argv[]);

namespace hpx {
inline int init(int argc, char* argv[]) {
    const int v = hpxhip_abi_version();
    if (v != HPXHIP_ABI_VERSION) {
        std::fprintf(stderr, "hpx::init: libhpxhip implements C ABI version %d, the headers expect %d\n", v,
                     HPXHIP_ABI_VERSION);
        return 1;
    }
    return hpx_main(argc, argv);
}
inline int finalize() { return 0; }
}  // namespace hpx
