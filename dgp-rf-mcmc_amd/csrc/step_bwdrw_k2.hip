// step_bwdrw_k2.hip — k_step_bwd_rw instances with KS = 2 A-tile k-steps (layer input width d <= 8).
#define DGPRF_KS 2
#include "step_bwdrw_impl.h"
