// tk_xsched.h -- which record slots go through which all-reduce (multi-rank), DESIGN.md 5.
//
// Every rank must issue the SAME sequence of all-reduces (same slot ranges, same element
// counts), or RCCL hangs or mixes records.  The schedule is therefore a pure function of
//   - the canonical call sequence: tk_decomp_init / step / sweep / flush / records /
//     basis_mul, which is the same on every rank of one job (the driver loop, with its
//     issue depth and worker count agreed over the ranks, tk_decomp_agree), and
//   - the group size, agreed at tk_decomp_create (element-wise max over the ranks),
// and never of rank-local state: how many factors a rank holds (none, for a rank beyond the
// factor count), whether its kernels defer a step's bookkeeping into the next launch
// (one-sweep) or not, its thread count, its timing.
//
// Slot s holds the record of step s-1 (slot 0: init).  Canonical events:
//   step_done(j)  end of tk_decomp_step(j): slots <= j become due (step j-1's record is
//                 written on every rank by then -- a one-sweep rank writes it in step j's
//                 launch); every full group of `group` due slots goes out as one all-reduce;
//   need(S)       a caller needs slots <= S exchanged now (records, sweep end, flush, a step
//                 with a record out): all unsent slots up to S go out as one all-reduce;
//   reset()       tk_decomp_init: a new sequence (unsent slots are dropped, never sent).
// Local completion (complete) is tracked only to refuse exchanging a slot this rank has
// not written yet.  No HIP here: tests/c/xsched_sim.cpp drives it on the CPU.
#ifndef TK_XSCHED_H_
#define TK_XSCHED_H_

#include <algorithm>
#include <utility>
#include <vector>

namespace tk {

struct XSched {
    typedef std::pair<int, int> Range;   // [first, last] slot, inclusive
    int group = 4;
    int sent = -1;    // slots <= sent are exchanged (this sequence)
    int due = -1;     // slots <= due are due
    int local = -1;   // slots <= local are written on this rank

    void reset() { sent = due = local = -1; }
    void complete(int s) { local = std::max(local, s); }
    bool written(int s) const { return s <= local; }

    // end of step j: the full groups to exchange now, in slot order
    std::vector<Range> step_done(int j) {
        std::vector<Range> out;
        due = std::max(due, j);
        while (due - sent >= group) {
            out.push_back(Range(sent + 1, sent + group));
            sent += group;
        }
        return out;
    }

    // slots (sent, S] now, as one range (first > last: nothing to send)
    Range need(int S) {
        if (S <= sent) return Range(1, 0);
        Range r(sent + 1, S);
        sent = S;
        due = std::max(due, S);
        return r;
    }
};

}  // namespace tk

#endif
