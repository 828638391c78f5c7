// step_bwdrw_k1.hip — k_step_bwd_rw instances with KS = 1 A-tile k-steps (layer input width d <= 4).
#define DGPRF_KS 1
#include "step_bwdrw_impl.h"
