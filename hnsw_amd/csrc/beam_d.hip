// beam_d.hip -- k_search_beam instantiations (beam.hpp) for 64x8, 64x12, 64x16
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<64, 8, 1>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 12, 1>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 16, 1>(const SearchArgs&, hipStream_t);
}  // namespace mh
