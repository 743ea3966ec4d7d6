/* ORACLE - test infrastructure only.  The float instantiation of the physics restatement (physics_oracle.c with
 * real = float; built with -fsingle-precision-constant so no literal widens an expression to double): the same
 * algorithm stepped in float32 arithmetic.  Its distance from the fp64 restatement over one env step is the
 * rounding error intrinsic to fp32 physics, the yardstick tests/test_gpu_scale.py holds the fp32 kernel to.
 * Exported: om_step_f32 (physics_oracle.c, public API section). */
#define OM_F32 1
#include "physics_oracle.c"
