// walks_b.hip -- k_search_compat / k_negatives instantiations (walks.hpp) for 64x2, 64x3
#include "walks.hpp"

namespace mh {
template int launch_compat_cfg<64, 2>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<64, 2>(const NegArgs&, hipStream_t);
template int launch_compat_cfg<64, 3>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<64, 3>(const NegArgs&, hipStream_t);
}  // namespace mh
