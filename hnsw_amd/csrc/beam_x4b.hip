// beam_x4b.hip -- k_search_beam instantiations (beam.hpp) with 4 entries expanded per
// layer-0 step (search_expand 4) for 64x4, 64x6, 64x8, 64x12, 64x16
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<64, 4, 4>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 6, 4>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 8, 4>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 12, 4>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 16, 4>(const SearchArgs&, hipStream_t);
}  // namespace mh
