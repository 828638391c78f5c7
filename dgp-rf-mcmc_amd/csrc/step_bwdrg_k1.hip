// step_bwdrg_k1.hip — k_step_bwd_rg instances with KS = 1 A-tile k-steps (layer input width d <= 4).
#define DGPRF_KS 1
#include "step_bwdrg_impl.h"
