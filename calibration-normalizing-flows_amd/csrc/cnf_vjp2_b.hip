// k_vjp2 instantiations, part B (cnf_vjp2.h): the packed-SGPR shapes of
// cnf_sgpr.hip's table, split over three translation units.
#include "cnf_vjp2.h"

namespace cnf {

const V2Entry kV2PartB[] = {
#ifdef CNF_VJP_DEV  // development builds: the headline shape only
    CNF_V2(10, 5, 5),
#else
    CNF_V2(3, 5, 0), CNF_V2(10, 5, 5), CNF_V2(3, 3, 3), CNF_V2(8, 3, 3), CNF_V2(10, 3, 3),
#endif
    {0, 0, 0, {}},  // sentinel (keeps the array non-empty in development builds)
};
const int kV2PartBNum = (int)(sizeof(kV2PartB) / sizeof(kV2PartB[0])) - 1;

}  // namespace cnf
