// local_rs.hip — instances of the packed LOCAL e-drift kernel (wavefront16.hpp) with u16 keys
// (WF16_LOCAL_U16) and the WITH_START reverse pass's early stop (WF16_LOCAL_RS,
// WF16_LOCAL_U16_RS) and with keys by step segments (WF16_LOCAL_SEG), over the packed shapes of dispatch.hip kShapes16.  Compiled apart from
// dispatch.hip so the two build in parallel.
#include <cstdlib>

#include "wavefront16.hpp"

namespace gx {

template <int ALGO>
static Wf16Fn pick(int G, int R) {
#define GX_CASE(g, r) if (G == g && R == r) return &wf16_kernel<ALGO, g, r>;
    GX_CASE(8, 8) GX_CASE(8, 12) GX_CASE(8, 16) GX_CASE(8, 19) GX_CASE(8, 20) GX_CASE(8, 23)
    GX_CASE(16, 10) GX_CASE(16, 12) GX_CASE(16, 16) GX_CASE(16, 20) GX_CASE(32, 5) GX_CASE(32, 6) GX_CASE(32, 9)
    GX_CASE(32, 20) GX_CASE(64, 3) GX_CASE(64, 5) GX_CASE(64, 20)
#undef GX_CASE
    return nullptr;
}

Wf16Fn wf16_local_lookup(int G, int R, bool u16, bool rs, bool seg) {
    // GASALX_KSEG_REG=1: the finished segments' per-row best in registers (A/B, VERDICT r05 item 6;
    // the instance of the 300 bp plan only)
    if (seg) {
        const char *e = std::getenv("GASALX_KSEG_REG");
        if (e && std::atoi(e) != 0 && G == 16 && R == 20) return &wf16_kernel<WF16_LOCAL_SEGR, 16, 20>;
        return pick<WF16_LOCAL_SEG>(G, R);
    }
    if (rs) return u16 ? pick<WF16_LOCAL_U16_RS>(G, R) : pick<WF16_LOCAL_RS>(G, R);
    return u16 ? pick<WF16_LOCAL_U16>(G, R) : pick<WF_LOCAL>(G, R);
}

}  // namespace gx
