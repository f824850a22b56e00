// k_vjp2 instantiations, part C (cnf_vjp2.h): the packed-SGPR shapes of
// cnf_sgpr.hip's table, split over three translation units.
#include "cnf_vjp2.h"

namespace cnf {

const V2Entry kV2PartC[] = {
#ifndef CNF_VJP_DEV
    CNF_V2(3, 3, 0), CNF_V2(3, 0, 0), CNF_V2(10, 0, 0), CNF_V2(10, 5, 0), CNF_V2(8, 5, 5),
#endif
    {0, 0, 0, {}},  // sentinel (keeps the array non-empty in development builds)
};
const int kV2PartCNum = (int)(sizeof(kV2PartC) / sizeof(kV2PartC[0])) - 1;

}  // namespace cnf
