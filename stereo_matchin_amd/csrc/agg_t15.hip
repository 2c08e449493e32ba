// aggregation passes for T = 15 taps (see asw_aggregate_impl.h)
#include "asw_aggregate_impl.h"
ASW_INSTANTIATE_PASS(15)
