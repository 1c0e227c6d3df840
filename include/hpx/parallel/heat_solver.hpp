// hpx/parallel/heat_solver.hpp -- the 1d_stencil heat solver over a
// partitioned_vector of HIP targets (one process, any number of partitions
// per target).
//
// Reference: examples/1d_stencil/1d_stencil_8.cpp:240-531 -- a `stepper`
// that owns partitions of the ring, and per time step computes every
// partition from its own points and one point of each neighbour
// (`heat_part`, 482-531, with the periodic neighbours of 1d_stencil_4_parallel.cpp:
// 147-150); U0[i] = i (1d_stencil_4.cpp:64-66), heat(l, m, r) =
// m + (k*dt/(dx*dx)) * (l - 2*m + r) (1d_stencil_1.cpp:41-46).
//
// Here a pass advances all partitions by S <= HPXHIP_STENCIL_MAX_FUSED steps
// at once (temporal blocking, hpxhip_stencil_heat_steps): each partition
// takes an S-point halo from each neighbour, copied device-to-device (peer
// copy across GPUs) into its own halo buffer on its own stream, so the ring
// exchanges once per S steps instead of once per step.  Results are
// bit-identical to S single steps (and to the serial example).
#pragma once

#include <hpx/components/containers/partitioned_vector/partitioned_vector.hpp>
#include <hpx/compute/hip.hpp>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace hpx { namespace compute { namespace hip {

class heat_solver {
public:
    using data_type = compute::vector<double, allocator<double>>;
    using space = partitioned_vector<double, data_type>;

    // 1d_stencil_8.cpp:290-300: nx points split into partitions (here: the
    // policy's layout over its targets), U0[i] = i
    explicit heat_solver(std::size_t nx, target_distribution_policy const& policy = target_layout, double k = 0.5,
                         double dt = 1.0, double dx = 1.0)
        : k_(k), dt_(dt), dx_(dx), u0_(nx, policy), u1_(nx, policy) {
        if (nx == 0) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "heat_solver: empty ring");
        std::vector<double> ramp(nx);
        for (std::size_t i = 0; i != nx; ++i) ramp[i] = static_cast<double>(i);
        set(ramp);
        for (std::size_t j = 0; j != u0_.get_num_partitions(); ++j) {
            auto const& p = u0_.get_partition(j);
            halo_.emplace_back(2 * HPXHIP_STENCIL_MAX_FUSED, allocator<double>(p.target));
        }
    }

    std::size_t size() const { return u0_.size(); }
    space const& current() const { return u(cur_); }

    // replace the state (nx values, host memory)
    void set(std::vector<double> const& values) {
        if (values.size() != size()) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "heat_solver: size");
        space& uc = u(cur_);
        for (std::size_t j = 0; j != uc.get_num_partitions(); ++j) {
            auto& p = uc.get_partition(j);
            if (p.last == p.first) continue;
            detail::check(hpxhip_memcpy_async(p.data->device_data(), values.data() + p.first, (p.last - p.first) * 8,
                                      HPXHIP_H2D, stream(j)),
                  "heat_solver: upload");
        }
        synchronize();
    }

    std::vector<double> to_host() const {
        std::vector<double> h(size());
        space const& uc = u(cur_);
        for (std::size_t j = 0; j != uc.get_num_partitions(); ++j) {
            auto const& p = uc.get_partition(j);
            if (p.last == p.first) continue;
            detail::check(hpxhip_memcpy_async(h.data() + p.first, p.data->device_data(), (p.last - p.first) * 8,
                                      HPXHIP_D2H, stream(j)),
                  "heat_solver: download");
        }
        const_cast<heat_solver*>(this)->synchronize();
        return h;
    }

    // stepper::do_work (1d_stencil_8.cpp:500-531): nt time steps
    space const& do_work(std::size_t nt) {
        std::size_t smallest = size();
        for (std::size_t j = 0; j != u0_.get_num_partitions(); ++j) {
            auto const& p = u0_.get_partition(j);
            if (p.last > p.first) smallest = std::min<std::size_t>(smallest, p.last - p.first);
        }
        while (nt > 0) {
            std::size_t s = std::min<std::size_t>({nt, std::size_t(HPXHIP_STENCIL_MAX_FUSED), smallest});
            if (s > 1 && (s & 1)) --s;  // the fused kernel takes 1 or an even count
            pass(static_cast<int>(s));
            nt -= s;
        }
        synchronize();
        return u(cur_);
    }

private:
    // Partition j of both buffers lives on one device, but each buffer's
    // partition holds its own target copy (and stream, cuda_target.cpp:
    // 203-211): all work on partition j goes to the stream of u0_'s copy, so
    // one synchronize() orders every pass.
    hpxhip_stream stream(std::size_t j) const { return u0_.get_partition(j).target.stream(); }
    void synchronize() {
        for (std::size_t j = 0; j != u0_.get_num_partitions(); ++j) u0_.get_partition(j).target.synchronize();
    }

    // the non-empty partition before / after j on the ring
    std::size_t neighbour(std::size_t j, bool left) const {
        const std::size_t np = u0_.get_num_partitions();
        for (std::size_t d = 1; d <= np; ++d) {
            const std::size_t q = left ? (j + np - d) % np : (j + d) % np;
            auto const& p = u0_.get_partition(q);
            if (p.last > p.first) return q;
        }
        return j;
    }

    // One pass of s steps.  Partition j's stream first waits, on the device,
    // for the previous pass of its two neighbours: their kernels wrote the
    // points j's halos copy now (RAW), and their halo copies read the points
    // j's kernel overwrites now (WAR).  The marks are all recorded before any
    // of this pass's work is queued, so a partition never waits for its
    // neighbours' new pass; no host wait between passes (r04 synchronised
    // every stream here).
    void pass(int s) {
        space& cur = u(cur_);
        space& nxt = u(cur_ ^ 1);
        const std::size_t np = cur.get_num_partitions();
        std::vector<detail::stream_mark> marks;
        marks.reserve(np);
        for (std::size_t j = 0; j != np; ++j) marks.emplace_back(stream(j));
        for (std::size_t j = 0; j != np; ++j) {
            auto& p = cur.get_partition(j);
            const uint64_t n = p.last - p.first;
            if (n == 0) continue;
            const std::size_t jl = neighbour(j, true), jr = neighbour(j, false);
            auto const& l = cur.get_partition(jl);
            auto const& r = cur.get_partition(jr);
            double* halo = halo_[j].device_data();
            const hpxhip_stream st = stream(j);
            marks[jl].wait_on(st);
            marks[jr].wait_on(st);
            // left halo = the left neighbour's last s points, right halo = the right neighbour's first s
            detail::check(hpxhip_memcpy_peer_async(halo, p.target.device(), l.data->device_data() + (l.last - l.first) - s,
                                           l.target.device(), 8 * static_cast<size_t>(s), st),
                  "heat_solver: halo");
            detail::check(hpxhip_memcpy_peer_async(halo + HPXHIP_STENCIL_MAX_FUSED, p.target.device(), r.data->device_data(),
                                           r.target.device(), 8 * static_cast<size_t>(s), st),
                  "heat_solver: halo");
            detail::check(hpxhip_stencil_heat_steps(p.data->device_data(), nxt.get_partition(j).data->device_data(), n, 0, n,
                                            halo, halo + HPXHIP_STENCIL_MAX_FUSED, s, k_, dt_, dx_, st),
                  "heat_solver: heat_part");
        }
        cur_ ^= 1;
    }

    space& u(int i) { return i ? u1_ : u0_; }
    space const& u(int i) const { return i ? u1_ : u0_; }

    double k_, dt_, dx_;
    space u0_, u1_;
    int cur_ = 0;
    std::vector<data_type> halo_;
};

}}}  // namespace hpx::compute::hip
