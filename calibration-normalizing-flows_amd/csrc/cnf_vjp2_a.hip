// k_vjp2 instantiations, part A (cnf_vjp2.h): the packed-SGPR shapes of
// cnf_sgpr.hip's table, split over three translation units.
#include "cnf_vjp2.h"

namespace cnf {

const V2Entry kV2PartA[] = {
#ifndef CNF_VJP_DEV
    CNF_V2(2, 5, 5), CNF_V2(3, 5, 5), CNF_V2(4, 5, 5), CNF_V2(5, 5, 5), CNF_V2(6, 5, 5),
#endif
    {0, 0, 0, {}},  // sentinel (keeps the array non-empty in development builds)
};
const int kV2PartANum = (int)(sizeof(kV2PartA) / sizeof(kV2PartA[0])) - 1;

}  // namespace cnf
