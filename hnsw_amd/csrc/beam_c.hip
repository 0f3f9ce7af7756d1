// beam_c.hip -- k_search_beam instantiations (beam.hpp) for 64x4, 64x6
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<64, 4, 1>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 6, 1>(const SearchArgs&, hipStream_t);
}  // namespace mh
