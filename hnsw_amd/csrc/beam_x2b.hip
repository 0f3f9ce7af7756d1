// beam_x2b.hip -- k_search_beam instantiations (beam.hpp) with 2 entries expanded per
// layer-0 step (search_expand 2) for 64x4, 64x6, 64x8, 64x12, 64x16
#include "beam.hpp"

namespace mh {
template int launch_beam_cfg<64, 4, 2>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 6, 2>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 8, 2>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 12, 2>(const SearchArgs&, hipStream_t);
template int launch_beam_cfg<64, 16, 2>(const SearchArgs&, hipStream_t);
}  // namespace mh
