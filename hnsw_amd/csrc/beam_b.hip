// beam_b.hip -- k_search_beam instantiations (beam.hpp) for 64x2, 64x3
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<64, 2, 1>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 3, 1>(const SearchArgs&, hipStream_t);
}  // namespace mh
