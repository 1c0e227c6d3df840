// hpx/components/containers/partitioned_vector/partitioned_vector.hpp --
// hpx::partitioned_vector over HIP targets in one process.
//
//   partitioned_vector<T, Data>      <- partitioned_vector_decl.hpp:146-405,
//                                       partitioned_vector_impl.hpp:317-395
//   hip::target_distribution_policy <- hpx/compute/cuda/target_distribution_policy.hpp:37-218,
//   hip::target_layout                  compute/detail/target_distribution_policy.hpp:79-131
//   segmented iterator               <- partitioned_vector_segmented_iterator.hpp:858-945
//
// This is the reference's CUDA configuration (examples/compute/cuda/
// partitioned_vector.cu: `partitioned_vector<int, compute::vector<int,
// cuda::allocator<int>>> v(1000, cuda::target_layout(get_local_targets()))`)
// with no AGAS: every partition is a compute::vector on one of the policy's
// targets.  N elements are split into k partitions of ceil(N/k)
// (partitioned_vector_impl.hpp:325, last shorter); partition j lives on
// target floor(j / ceil(k / T)) -- contiguous runs of partitions per target,
// in target order, as bulk_create hands them out (default_distribution_
// policy.hpp:294-324, with its degenerate counts for k < T clipped instead).
//
// The segmented algorithms over these iterators are in
// <hpx/parallel/segmented_algorithms.hpp> (included by hpx/hpx.hpp).
#pragma once

#include <hpx/compute/hip.hpp>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <iterator>
#include <memory>
#include <stdexcept>
#include <type_traits>
#include <vector>

namespace hpx {
namespace compute { namespace hip {

struct target_distribution_policy {
    std::vector<target> targets;
    std::size_t num_partitions = std::size_t(-1);

    target_distribution_policy() = default;
    target_distribution_policy(std::vector<target> ts, std::size_t k) : targets(std::move(ts)), num_partitions(k) {}

    // target_distribution_policy.hpp:53-62 / 84-92
    target_distribution_policy operator()(std::vector<target> const& ts,
                                          std::size_t k = std::size_t(-1)) const {
        return target_distribution_policy(ts, k == std::size_t(-1) ? ts.size() : k);
    }
    target_distribution_policy operator()(target const& t, std::size_t k = 1) const {
        return target_distribution_policy(std::vector<target>{t}, k);
    }

    std::vector<target> const& get_targets() const { return targets; }
    // compute/detail/target_distribution_policy.hpp:88-96: default = one per target, at least one
    std::size_t get_num_partitions(std::size_t ntargets) const {
        std::size_t k = num_partitions == std::size_t(-1) ? ntargets : num_partitions;
        return k < 1 ? 1 : k;
    }
};

// hpx::compute::cuda::target_layout
inline target_distribution_policy const target_layout{};

}}  // namespace compute::hip

template <typename T, typename Data = compute::vector<T, compute::hip::allocator<T>>>
class partitioned_vector;

template <typename PV>
class partitioned_vector_iterator {
    PV* pv_ = nullptr;
    std::size_t pos_ = 0;

public:
    using iterator_category = std::random_access_iterator_tag;
    using value_type = typename PV::value_type;
    using difference_type = std::ptrdiff_t;
    using pointer = void;
    using reference = compute::hip::value_proxy<value_type>;
    using container_type = PV;

    partitioned_vector_iterator() = default;
    partitioned_vector_iterator(PV* pv, std::size_t pos) : pv_(pv), pos_(pos) {}
    PV& container() const { return *pv_; }
    std::size_t index() const { return pos_; }

    reference operator*() const { return (*pv_)[pos_]; }
    reference operator[](difference_type i) const { return (*pv_)[pos_ + i]; }
    partitioned_vector_iterator& operator++() { ++pos_; return *this; }
    partitioned_vector_iterator operator++(int) { auto r = *this; ++pos_; return r; }
    partitioned_vector_iterator& operator--() { --pos_; return *this; }
    partitioned_vector_iterator& operator+=(difference_type n) { pos_ += n; return *this; }
    partitioned_vector_iterator& operator-=(difference_type n) { pos_ -= n; return *this; }
    friend partitioned_vector_iterator operator+(partitioned_vector_iterator a, difference_type n) { return a += n; }
    friend partitioned_vector_iterator operator-(partitioned_vector_iterator a, difference_type n) { return a -= n; }
    friend difference_type operator-(partitioned_vector_iterator const& a, partitioned_vector_iterator const& b) {
        return static_cast<difference_type>(a.pos_) - static_cast<difference_type>(b.pos_);
    }
    friend bool operator==(partitioned_vector_iterator const& a, partitioned_vector_iterator const& b) {
        return a.pv_ == b.pv_ && a.pos_ == b.pos_;
    }
    friend bool operator!=(partitioned_vector_iterator const& a, partitioned_vector_iterator const& b) {
        return !(a == b);
    }
};

template <typename It>
struct is_segmented_iterator : std::false_type {};
template <typename PV>
struct is_segmented_iterator<partitioned_vector_iterator<PV>> : std::true_type {};

template <typename T, typename Data>
class partitioned_vector {
public:
    using value_type = T;
    using data_type = Data;
    using allocator_type = typename Data::allocator_type;
    using iterator = partitioned_vector_iterator<partitioned_vector>;
    using const_iterator = iterator;

    struct partition {
        std::size_t first = 0, last = 0;  // global [first, last)
        compute::hip::target target;
        std::unique_ptr<Data> data;
    };

    explicit partitioned_vector(std::size_t n,
                                compute::hip::target_distribution_policy const& policy = compute::hip::target_layout)
        : size_(n) {
        create(policy, nullptr);
    }
    partitioned_vector(std::size_t n, T const& v,
                       compute::hip::target_distribution_policy const& policy = compute::hip::target_layout)
        : size_(n) {
        create(policy, &v);
    }
    partitioned_vector(partitioned_vector const&) = delete;
    partitioned_vector& operator=(partitioned_vector const&) = delete;

    std::size_t size() const { return size_; }
    bool empty() const { return size_ == 0; }
    std::size_t get_num_partitions() const { return parts_.size(); }
    partition const& get_partition(std::size_t j) const { return parts_[j]; }
    partition& get_partition(std::size_t j) { return parts_[j]; }
    // index of the partition holding global element i (partitions of ceil(N/k))
    std::size_t partition_of(std::size_t i) const { return part_size_ ? i / part_size_ : 0; }

    // the device data is not const-protected (compute::vector's iterators
    // are not either): const containers hand out the same iterators
    iterator begin() const { return iterator(const_cast<partitioned_vector*>(this), 0); }
    iterator end() const { return iterator(const_cast<partitioned_vector*>(this), size_); }

    compute::hip::value_proxy<T> operator[](std::size_t i) {
        partition& p = parts_[partition_of(i)];
        return (*p.data)[i - p.first];
    }

private:
    void create(compute::hip::target_distribution_policy const& policy, T const* v) {
        std::vector<compute::hip::target> ts = policy.get_targets();
        if (ts.empty()) ts = compute::hip::get_local_targets();
        if (ts.empty()) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "partitioned_vector: no HIP targets");
        const std::size_t k = policy.get_num_partitions(ts.size());
        part_size_ = (size_ + k - 1) / k;  // partitioned_vector_impl.hpp:325
        const std::size_t run = (k + ts.size() - 1) / ts.size();
        parts_.resize(k);
        for (std::size_t j = 0; j < k; ++j) {
            partition& p = parts_[j];
            p.first = std::min(size_, j * part_size_);
            p.last = std::min(size_, p.first + part_size_);
            p.target = ts[std::min(ts.size() - 1, j / run)];
            compute::hip::allocator<T> alloc(p.target);
            p.data = v ? std::make_unique<Data>(p.last - p.first, *v, alloc)
                       : std::make_unique<Data>(p.last - p.first, alloc);
        }
    }

    std::size_t size_ = 0;
    std::size_t part_size_ = 0;
    std::vector<partition> parts_;
};

}  // namespace hpx
