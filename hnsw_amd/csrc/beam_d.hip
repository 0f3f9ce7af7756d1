// beam_d.hip -- k_search_beam instantiations (beam.hpp) for 64x8, 64x12, 64x16
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<64, 8>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 12>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 16>(const SearchArgs&, hipStream_t);
}  // namespace mh
