// hpx/parallel/segmented_fwd.hpp -- declarations of the segmented algorithms
// (definitions: <hpx/parallel/segmented_algorithms.hpp>) so that the
// algorithms of <hpx/parallel/algorithms.hpp> can hand partitioned_vector
// iterators over to them (the reference dispatches on the iterator's
// segmented trait the same way, e.g. for_each.hpp:540-552 -> for_each_ with
// is_segmented_iterator, segmented_algorithms/for_each.hpp:197-213).
#pragma once

#include <hpx/components/containers/partitioned_vector/partitioned_vector.hpp>
#include <hpx/parallel/execution.hpp>

namespace hpx { namespace parallel { inline namespace v1 { namespace segmented_detail {

template <typename P, typename It, typename F>
typename util::detail::algorithm_result<P, It>::type for_each(P&& p, It first, It last, F&& f);

template <typename P, typename It, typename T>
typename util::detail::algorithm_result<P, void>::type fill(P&& p, It first, It last, T const& value);

template <typename P, typename In, typename Out, typename F>
typename util::detail::algorithm_result<P, util::tagged_pair<In, Out>>::type transform(P&& p, In first, In last,
                                                                                      Out dest, F&& f);

template <typename P, typename In1, typename In2, typename Out, typename F>
typename util::detail::algorithm_result<P, util::tagged_tuple<In1, In2, Out>>::type transform_binary(
    P&& p, In1 first1, std::size_t n, In2 first2, Out dest, F&& f);

template <typename T, typename P, typename It, typename Op, typename Conv>
typename util::detail::algorithm_result<P, T>::type reduce(P&& p, It first, It last, T init, Op&& op, Conv&& conv);

template <typename P, typename In, typename Out, typename Op, typename Conv, typename T>
typename util::detail::algorithm_result<P, Out>::type scan(P&& p, In first, In last, Out dest, Op&& op, Conv&& conv,
                                                          T init, bool inclusive);

template <typename P, typename In, typename Out>
typename util::detail::algorithm_result<P, util::tagged_pair<In, Out>>::type copy(P&& p, In first, In last,
                                                                                 Out dest);

}}}}  // namespace hpx::parallel::v1::segmented_detail
