// cimq_part_v7_33.hip -- the v7 backward for w3a3 layers (nbw = nba = 3).
#include "cimq_v7_launch.h"

namespace cimq {
template CIMQ_V7_SIG(3, 3);
}  // namespace cimq
