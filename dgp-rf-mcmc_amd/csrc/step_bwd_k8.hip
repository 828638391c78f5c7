// step_bwd_k8.hip — k_step_bwd instances with KS = 8 A-tile k-steps (layer input width d <= 32).
#define DGPRF_KS 8
#include "step_bwd_impl.h"
