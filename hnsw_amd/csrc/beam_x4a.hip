// beam_x4a.hip -- k_search_beam instantiations (beam.hpp) with 4 entries expanded per
// layer-0 step (search_expand 4) for 16x1, 32x1, 64x1, 64x2, 64x3
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<16, 1, 4>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<32, 1, 4>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 1, 4>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 2, 4>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 3, 4>(const SearchArgs&, hipStream_t);
}  // namespace mh
