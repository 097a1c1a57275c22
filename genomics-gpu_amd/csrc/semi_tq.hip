// semi_tq.hip — instances of the packed SEMI-GLOBAL kernel for TAIL = QUERY / BOTH
// (wavefront16.hpp, WF16_SEMI_TQ): one per padded target length 8R, R = 1..32, so
// that a class launch's last padded column is register R - 1 of lane 7.  Compiled
// apart from dispatch.hip so the two build in parallel.
#include "wavefront16.hpp"

namespace gx {

template <int R> static Wf16Fn tq() { return &wf16_kernel<WF16_SEMI_TQ, 8, R>; }

template <int... Rs> static Wf16Fn tq_pick(int R, std::integer_sequence<int, Rs...>) {
    Wf16Fn out = nullptr;
    ((R == Rs + 1 ? (out = tq<Rs + 1>(), 0) : 0), ...);
    return out;
}

Wf16Fn wf16_tq_lookup(int R) { return tq_pick(R, std::make_integer_sequence<int, 32>{}); }

}  // namespace gx
