"""The exact per-key rule of C4's shape for ANY timestamp order (test infrastructure, CPU).

`every (e1=S1[f] and e2=S2[f]) -> not S3[fz(e1, z)] for T within W` in playback, restated from the
processors the oracle restates (oracle/oracle.cpp, each step citing the reference):

per partition key
  partial   the logical partial: an x (e1) slot and a y (e2) slot (LogicalPreStateProcessor; one at a
            time: `every` re-arms a fresh one when it completes or expires)
  pend/nae  the pairs on the absent state's pending / new-and-every lists, in list order
            (AbsentStreamPreStateProcessor.addState appends to new-and-every; updateState moves
            them, stably sorted by ts, StreamPreStateProcessor.java:308-323)
  fifo      the Scheduler's ToNotifyQueue of this key: timer entries in insertion order (a FIFO,
            Scheduler.java:113-127, 332), each with the first batch index it may fire at
  lst       AbsentStreamPreStateProcessor's lastScheduledTime

playback clock: a send whose clock is >= the app clock sets it and fires every timer entry at the
head of a queue that the clock reached (TimestampGeneratorImpl.setCurrentTimestamp :105-121,
Scheduler.onTimeChange :71-103, sendTimerEvents :171-209); a send below the clock fires none.

timer entry e firing at batch index g (AbsentStreamPreStateProcessor.process :151-227):
  new-and-every -> pending; every pending pair expired at e (|slot ts - e| > W) is dropped, every
  pair with e >= its ts + T is emitted (ts = e) in list order; lst = clock + T when the clock passed
  e + T; nothing emitted and lst < e -> lst = e + T and a new entry e + T (the re-arm).
key event at t (stabilizeStates then processAndReturn, oracle Engine.sendEvent):
  expireEvents (every pre, ts t): a logical partial with a filled slot more than W from t re-arms;
  the absent pending list drops expired pairs from its head (stopping at the first live one), its
  new-and-every list every expired pair (StreamPreStateProcessor.expireEvents :326-361);
  Z: new-and-every -> pending, then each pending pair whose fz holds is dropped, and each drop sets
  lst = t + T and queues an entry t + T (AbsentStreamPostStateProcessor.process :36-56 ->
  updateLastArrivalTime :68-78);
  X / Y with its filter: fills its slot if empty (LogicalPreStateProcessor.processAndReturn
  :128-167); with the partner filled the pair completes: it joins new-and-every with ts t, lst =
  t + T, an entry t + T is queued (AbsentStreamPreStateProcessor.addState :80-103), and the partial
  re-arms (LogicalPostStateProcessor.process :59-87).
Cross-key ties of onTimeChange's TreeMultimap (one key per distinct due time per call) are not
modelled (parity-unpinned); the tests' streams have none.

labs.h's k_labs (a thread per key) implements exactly this; k_labs_w (a wave per key) implements
its ordered special case (`wave_exact` in tests/test_labs.py checks that they agree, state included).
"""
from __future__ import annotations

import bisect
from collections import deque

import numpy as np

W, WAIT = 10_000, 5_000


class KeyState:
    __slots__ = ("x", "y", "pend", "nae", "fifo", "lst", "last", "gfired")

    def __init__(self):
        self.x = self.y = None   # (seq, ts, value)
        self.pend = []           # pairs: (x, y, ts)
        self.nae = []
        self.fifo = deque()      # (time, first batch index it may fire at)
        self.lst = 0
        self.last = None         # ts of the key's latest event
        self.gfired = 0          # batch index of the push's latest firing of this key's queue

    def snapshot(self):
        """The state as plain data (pairs as (xseq, yseq, ts), entries as times)."""
        return ((self.x[0] if self.x else -1, self.y[0] if self.y else -1),
                tuple((p[0][0], p[1][0], p[2]) for p in self.pend),
                tuple((p[0][0], p[1][0], p[2]) for p in self.nae),
                tuple(e for e, _ in self.fifo), self.lst)


def _stable_ts(pairs):
    return sorted(pairs, key=lambda p: p[2])  # eventTimeComparator, stable (no ts -1 here)


class ExactC4:
    """Runs pushes of (ts, key, stream, price[, clock]) and collects records per key:
    (ts, type, pos, ((y seq,), (x seq,), ())) -- the slot order of program_for(4) (state 0 = e2)."""

    def __init__(self, W=W, T=WAIT, fz=lambda z, x, y: z > x, start_clock=0):
        self.W, self.T, self.fz = W, T, fz
        self.keys = {}
        self.clock = start_clock
        self.seq = 0
        self.out = {}
        self.rearms = 0
        self.jumps = 0

    def _fire(self, k, K, upto, rmax, nxf, base):
        """Fire k's queue heads whose firing event is at or before batch index `upto`."""
        T, W = self.T, self.W
        while K.fifo:
            e, i0 = K.fifo[0]
            i0 = max(i0, K.gfired)  # a FIFO: no entry fires before the one ahead of it
            lb = bisect.bisect_left(rmax, e, lo=i0)
            g = max(lb, nxf[i0]) if i0 < len(rmax) else len(rmax)
            if g > upto:
                return
            K.fifo.popleft()
            K.gfired = g
            actual = rmax[g]
            K.pend += _stable_ts(K.nae)
            K.nae = []
            keep, ret = [], []
            for p in K.pend:
                if W >= 0 and (abs(p[0][1] - e) > W or abs(p[1][1] - e) > W):
                    continue
                if e >= p[2] + T:
                    ret.append(p)
                    continue
                keep.append(p)
            K.pend = keep
            for p in ret:
                self.out.setdefault(k, []).append((e, 0, base + g, ((p[1][0],), (p[0][0],), ())))
            if actual > T + e:
                K.lst = actual + T
                self.jumps += 1
            if not ret and K.lst < e:
                K.lst = e + T
                K.fifo.append((e + T, g))
                self.rearms += 1

    def push(self, ts, key, st, pr, clk=None):
        ts = np.asarray(ts, np.int64)
        clk = ts if clk is None else np.asarray(clk, np.int64)
        n = len(ts)
        base = self.seq
        rmax = np.maximum.accumulate(np.concatenate([[self.clock], clk]))[1:]
        prev = np.concatenate([[self.clock], rmax[:-1]])
        firing = clk >= prev
        nxf = np.full(n + 1, n, np.int64)  # first firing index >= g
        for g in range(n - 1, -1, -1):
            nxf[g] = g if firing[g] else nxf[g + 1]
        rm = rmax.tolist()
        nxl = nxf.tolist()
        W, T = self.W, self.T
        for q in range(n):
            s = int(st[q])
            if s < 0:
                continue
            k = int(key[q])
            K = self.keys.get(k)
            if K is None:
                K = self.keys[k] = KeyState()
            self._fire(k, K, q, rm, nxl, base)
            t, v = int(ts[q]), float(pr[q])
            K.last = t
            # expireEvents: the logical partial, then the absent lists
            if W >= 0 and ((K.x and abs(K.x[1] - t) > W) or (K.y and abs(K.y[1] - t) > W)):
                K.x = K.y = None
            while K.pend and W >= 0 and (abs(K.pend[0][0][1] - t) > W or abs(K.pend[0][1][1] - t) > W):
                K.pend.pop(0)
            if W >= 0:
                K.nae = [p for p in K.nae if not (abs(p[0][1] - t) > W or abs(p[1][1] - t) > W)]
            ev = (base + q, t, v)
            if s == 2:
                K.pend += _stable_ts(K.nae)
                K.nae = []
                keep = []
                for p in K.pend:
                    if self.fz(v, p[0][2], p[1][2]):
                        K.lst = t + T
                        K.fifo.append((t + T, q + 1))
                    else:
                        keep.append(p)
                K.pend = keep
            elif v > 20:
                if s == 0 and K.x is None:
                    K.x = ev
                elif s == 1 and K.y is None:
                    K.y = ev
                else:
                    continue
                if K.x is not None and K.y is not None:
                    K.nae.append((K.x, K.y, t))
                    K.lst = t + T
                    K.fifo.append((t + T, q + 1))
                    K.x = K.y = None
        for k, K in self.keys.items():  # the timers the push's last clock reaches
            self._fire(k, K, n - 1, rm, nxl, base)
        # the queue entries carry over: indices restart at the next push
        for K in self.keys.values():
            K.fifo = deque((e, 0) for e, _ in K.fifo)
            K.gfired = 0
        if n:
            self.clock = int(rmax[-1])
        self.seq += n

    def fetch(self):
        out, self.out = self.out, {}
        return out


class FastC4:
    """The ordered special case k_labs_w implements, as formulas per pair rather than an event loop
    over the absent state (test infrastructure).  Valid for a push when every key's timestamps do
    not decrease, no key event lags the clock by T or more, the clock never steps by more than T,
    and every key's state is regular (queue sorted, lst >= its last entry <= last ts + T, pairs in
    ts order).  Then per pair P (completed at key event c, slots' earliest ts m, due = c + T, D =
    m + W): the queue is always sorted, every entry <= the clock has fired, and
      E_D   = min(due, the first queue entry > max(D, clock(c)) present at c): P leaves the pending
              list (fires if due <= D, else silently expires) before the first key event q > c with
              clock(q) >= E_D or ts(q) > D, or at the push's end if the last clock reaches E_D;
      kill  = the first Z event in (c, that q) whose fz holds: the kill queues an entry ts + T;
      H     = the queue's head at c: P is still on new-and-every at the end iff no Z event of the
              key came after c and H > the last clock;
    lst is ts + T of the key's last completion or kill; the queue keeps every entry > the last clock.
    Must equal ExactC4, outputs and state (tests/test_labs.py)."""

    def __init__(self, W=W, T=WAIT, fz=lambda z, x, y: z > x, start_clock=0):
        self.W, self.T, self.fz = W, T, fz
        self.keys = {}
        self.clock = start_clock
        self.seq = 0
        self.out = {}

    def push(self, ts, key, st, pr):
        ts = np.asarray(ts, np.int64)
        n = len(ts)
        base = self.seq
        rmax = np.maximum.accumulate(np.concatenate([[self.clock], ts]))[1:]
        prevc = self.clock
        W, T = self.W, self.T
        Wn = W if W >= 0 else 1 << 62
        # validity (else the exact kernel runs the push)
        steps = np.diff(np.concatenate([[self.clock], rmax]))
        if n and not any(K["fifo"] for K in self.keys.values()):
            steps[0] = 0  # nothing is queued yet: the first step fires no entry
        if n and steps.max() > T:
            raise ValueError("clock step > T")
        runs = {}
        for q in range(n):
            if int(st[q]) >= 0:
                runs.setdefault(int(key[q]), []).append(q)
        clk_end = int(rmax[-1]) if n else self.clock
        for k in set(runs) | set(self.keys):
            K = self.keys.get(k)
            if K is None:
                K = self.keys[k] = {"x": None, "y": None, "pairs": [], "fifo": [], "lst": 0, "last": None,
                                    "nae": 0}
            idx = runs.get(k, [])
            fifo = list(K["fifo"])  # (time, creation index): carried entries created before the push
            fifo = [(e, -1) for e in fifo]
            pairs = [dict(p, c=-1, was_nae=(i >= len(K["pairs"]) - K["nae"])) for i, p in enumerate(K["pairs"])]
            lastZ, lst_pos, lst = -1, -2, K["lst"]
            for q in idx:
                t = int(ts[q])
                if K["last"] is not None and t < K["last"]:
                    raise ValueError("decrease")
                if int(rmax[q]) - t >= T:
                    raise ValueError("lag")
                K["last"] = t
            # the logical partial and completions (as labs.h's pend rule)
            x, y = K["x"], K["y"]
            for q in idx:
                t, s, v = int(ts[q]), int(st[q]), float(pr[q])
                if (x and abs(x[1] - t) > W and W >= 0) or (y and abs(y[1] - t) > W and W >= 0):
                    x = y = None
                if s == 2:
                    lastZ = q
                    continue
                if v <= 20:
                    continue
                if s == 0 and x is None:
                    x = (base + q, t, v)
                elif s == 1 and y is None:
                    y = (base + q, t, v)
                else:
                    continue
                if x and y:
                    pairs.append({"x": x, "y": y, "ts": t, "c": q, "was_nae": True})
                    x = y = None
            K["x"], K["y"] = x, y
            # per pair in completion order: E_D, H, fate
            new_entries = []  # (time, creation index)
            for p in pairs:
                c = p["c"]
                due = p["ts"] + T
                D = min(p["x"][1], p["y"][1]) + Wn
                if c >= 0:  # completed in this push: the queue at c
                    cc = int(rmax[c])
                    present = [e for e, i in fifo + new_entries if i < c and e > cc]
                    p["H"] = min(present + [due])
                    cand = [e for e in present if e > max(D, cc)]
                    p["ED"] = min(cand + [due])
                    new_entries.append((due, c))
                ED = p["ED"]
                lo = c + 1 if c >= 0 else 0
                later = [q for q in idx if q >= lo]
                fq = next((q for q in later if int(rmax[q]) >= ED or int(ts[q]) > D), None)
                kill = next((q for q in later if (fq is None or q < fq) and int(st[q]) == 2
                             and self.fz(float(pr[q]), p["x"][2], p["y"][2])), None)
                p["dead"] = False
                if kill is not None:
                    new_entries.append((int(ts[kill]) + T, kill))
                    if kill > lst_pos:
                        lst_pos, lst = kill, int(ts[kill]) + T
                    p["dead"] = True
                elif fq is not None or clk_end >= ED:
                    if due <= D:  # fires: the first firing event at or after its due
                        g = int(np.searchsorted(rmax, due, side="left"))
                        g = max(g, lo if c >= 0 else 0)
                        self.out.setdefault(k, []).append((due, 0, base + g, ((p["y"][0],), (p["x"][0],), ())))
                    p["dead"] = True
                if c >= 0 and c > lst_pos:
                    lst_pos, lst = c, int(ts[c]) + T
            alive = [p for p in pairs if not p["dead"]]
            # records of one key in fire order: pairs fire in completion order
            K["pairs"] = [{k2: p[k2] for k2 in ("x", "y", "ts", "H", "ED")} for p in alive]
            nae = 0
            for p in reversed(alive):
                if (p["was_nae"] and p["c"] >= lastZ) and p["H"] > clk_end:
                    nae += 1
                else:
                    break
            K["nae"] = nae
            K["fifo"] = sorted(e for e, _ in fifo + new_entries if e > clk_end)
            K["lst"] = lst
        if n:
            self.clock = clk_end
        self.seq += n

    def state(self, k):
        K = self.keys[k]
        pend = K["pairs"][:len(K["pairs"]) - K["nae"]]
        nae = K["pairs"][len(K["pairs"]) - K["nae"]:]
        return ((K["x"][0] if K["x"] else -1, K["y"][0] if K["y"] else -1),
                tuple((p["x"][0], p["y"][0], p["ts"]) for p in pend),
                tuple((p["x"][0], p["y"][0], p["ts"]) for p in nae), tuple(K["fifo"]), K["lst"])

    def fetch(self):
        out, self.out = self.out, {}
        return out
