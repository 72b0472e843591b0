// ORACLE — test infrastructure only (see common.hpp header).
//
// Elementary functions used by the restatement. Default: detmath (the
// deterministic library the HIP kernels also use, detmath/detmath.h), so the
// oracle is a bit-exact checker for the GPU path. Built with -DORACLE_LIBM the
// oracle uses the host libm instead, as the reference build does; tests compare
// the two variants to bound the effect of the elementary-function library.
// The incomplete gamma (boost::math::gamma_p in the reference) always comes
// from detmath::gamma_pq, evaluated with this build's exp/log.
//
// The reference writes every power as std::pow. The detmath build evaluates
// the small integer powers by squaring (OPOW4, OPOW8) and the fractional powers
// of moderate arguments and odeint's step-size controller as exp(y log x)
// (OPOWR); the libm build keeps std::pow for all of them.
#pragma once
#include <cmath>

#include "../../detmath/detmath.h"

#ifdef ORACLE_LIBM
#define OEXP(x) std::exp(x)
#define OLOG(x) std::log(x)
#define OPOW(x, y) std::pow(x, y)
#define OPOW4(x) std::pow(x, 4)
#define OPOW8(x) std::pow(x, 8)
#define OPOWR(x, y) std::pow(x, y)
#define OLGAMMA(x) std::lgamma(x)
#else
#define OEXP(x) detmath::exp(x)
#define OLOG(x) detmath::log(x)
#define OPOW(x, y) detmath::pow((double)(x), (double)(y))
#define OPOW4(x) detmath::pow4((double)(x))
#define OPOW8(x) detmath::pow8((double)(x))
#define OPOWR(x, y) detmath::powr((double)(x), (double)(y))
#define OLGAMMA(x) detmath::lgamma(x)
#endif
