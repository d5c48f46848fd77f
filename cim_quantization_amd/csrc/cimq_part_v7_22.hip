// cimq_part_v7_22.hip -- the v7 backward for w2a2 layers (nbw = nba = 2).
#include "cimq_v7_launch.h"

namespace cimq {
template CIMQ_V7_SIG(2, 2);
}  // namespace cimq
