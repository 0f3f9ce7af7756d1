// beam_x2a.hip -- k_search_beam instantiations (beam.hpp) with 2 entries expanded per
// layer-0 step (search_expand 2) for 16x1, 32x1, 64x1, 64x2, 64x3
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<16, 1, 2>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<32, 1, 2>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 1, 2>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 2, 2>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 3, 2>(const SearchArgs&, hipStream_t);
}  // namespace mh
