// walks_c.hip -- k_search_compat / k_negatives instantiations (walks.hpp) for 64x4, 64x6
#include "walks.hpp"

namespace mh {
template int launch_compat_cfg<64, 4>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<64, 4>(const NegArgs&, hipStream_t);
template int launch_compat_cfg<64, 6>(const SearchArgs&, hipStream_t);
template int launch_negatives_cfg<64, 6>(const NegArgs&, hipStream_t);
}  // namespace mh
