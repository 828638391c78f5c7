// step_fwd_k1.hip — k_step_fwd instances with KS = 1 A-tile k-steps (layer input width d <= 4).
#define DGPRF_KS 1
#include "step_fwd_impl.h"
