// hpx/hpx_init.hpp -- HPX's explicit start-up shape (hpx::init runs the
// user's hpx_main, hpx::finalize ends it; hpx/hpx_init.hpp in HPX 1.4.0).
// The HIP backend has no AGAS/thread-manager to boot: init calls hpx_main
// on the calling thread and returns its result.
#pragma once

int hpx_main(int argc, char* argv[]);

namespace hpx {
inline int init(int argc, char* argv[]) { return hpx_main(argc, argv); }
inline int finalize() { return 0; }
}  // namespace hpx
