// beam_a.hip -- k_search_beam instantiations (beam.hpp) for 16x1, 32x1, 64x1
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<16, 1, 1>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<32, 1, 1>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 1, 1>(const SearchArgs&, hipStream_t);
}  // namespace mh
