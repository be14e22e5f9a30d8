// The wide instance of the g2o-order LocalBundleAdjustment (lba_g2o.hip with two-word pose masks: up to 128 free
// poses, reduced systems up to 768 rows), run for windows of more than 64 keyframes; lba_run_g2o picks the instance.
#define LBG_PW 2
#include "lba_g2o.hip"
