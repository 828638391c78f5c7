// step_bwdrg_k0.hip — k_step_bwd_rg instances with KS = 0 A-tile k-steps (d > 32: A_1 precomputed).
#define DGPRF_KS 0
#include "step_bwdrg_impl.h"
