// walks_a.hip -- k_search_compat / k_negatives instantiations (walks.hpp) for 16x1, 32x1, 64x1
#include "walks.hpp"

namespace mh {
template int launch_compat_cfg<16, 1>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<16, 1>(const NegArgs&, hipStream_t);
template int launch_compat_cfg<32, 1>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<32, 1>(const NegArgs&, hipStream_t);
template int launch_compat_cfg<64, 1>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<64, 1>(const NegArgs&, hipStream_t);
}  // namespace mh
