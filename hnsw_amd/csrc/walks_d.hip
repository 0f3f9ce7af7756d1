// walks_d.hip -- k_search_compat / k_negatives instantiations (walks.hpp) for 64x8, 64x12, 64x16
#include "walks.hpp"

namespace mh {
template int launch_compat_cfg<64, 8>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<64, 8>(const NegArgs&, hipStream_t);
template int launch_compat_cfg<64, 12>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<64, 12>(const NegArgs&, hipStream_t);
template int launch_compat_cfg<64, 16>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<64, 16>(const NegArgs&, hipStream_t);
}  // namespace mh
