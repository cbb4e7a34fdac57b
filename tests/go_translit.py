"""TEST INFRASTRUCTURE ONLY — a second, independent restatement of the hot path (A1–A5).

The Go reference cannot run here (no Go toolchain) and ships no vectors for this path, so parity
rests on restatements of its text. oracle/oracle.cpp is one (record-at-a-time C over the engine's
flat records). This module is another, written separately and shaped differently on purpose: a
literal transliteration of the cited Go functions over Go-shaped objects (an instanceSpace of
*Instance with a LeaderBookkeeping, a PrepareBookkeeping, a State whose Store is a map), with
panics raised where Go would panic. Only the adapter class GoBackend at the bottom knows the
engine's record layouts; it converts them into those objects and back. A misreading of the Go in
one restatement shows up as a disagreement with the other (tests/test_go_translit.py runs both on
every golden fixture, the known-answer cases and seeded random batches).

Where the engine's batch contract has to say something the Go leaves implicit, the adapter says
it (marked CONTRACT): the instance window is the slice, a nil instance stops the execute cursor,
group tables keep Go-map insertion order.
"""
import numpy as np

from minpaxos_amd import records as R

TRUE = 1  # bareminpaxos.go:19, paxos.go `const TRUE = uint8(1)`

# minpaxosproto.InstanceStatus / paxos InstanceStatus (minpaxosproto.go:8-15, paxos.go:35-41)
PREPARING, PREPARED, ACCEPTED, COMMITTED = 0, 1, 2, 3

# state.Operation (state.go:10-19)
NONE, PUT, GET, DELETE, RLOCK, WLOCK = 0, 1, 2, 3, 4, 5
NIL = 0  # state.go:23


class GoPanic(Exception):
    """runtime panic (index out of range / nil pointer dereference)"""

    def __init__(self, code, what):
        super().__init__(what)
        self.code = code


def i32(x):
    """int32 arithmetic wraps as in Go"""
    return (x + (1 << 31)) % (1 << 32) - (1 << 31)


class Slice:
    """a Go slice indexed from `base` (the instance window handed to the batch call)"""

    def __init__(self, base, items):
        self.base, self.items = base, items

    def _at(self, i):
        j = i - self.base
        if j < 0 or j >= len(self.items):
            raise GoPanic(R.E_NIL_INSTANCE, f"index {i} out of range")
        return j

    def __getitem__(self, i):
        return self.items[self._at(i)]

    def __setitem__(self, i, v):
        self.items[self._at(i)] = v

    def get_or_nil(self, i):
        """CONTRACT: instances past the window do not exist yet (nil)"""
        j = i - self.base
        return self.items[j] if 0 <= j < len(self.items) else None


def setidx(arr, i, v):
    """arr[i] = v with Go's bounds check"""
    if i < 0 or i >= len(arr):
        raise GoPanic(R.E_BAD_ID, f"index {i} out of range [0:{len(arr)}]")
    arr[i] = v


def deref(p, what):
    if p is None:
        raise GoPanic(R.E_NIL_INSTANCE, f"nil pointer dereference ({what})")
    return p


# ---- package state  src/state/state.go ----------------------------------------------------------
class Command:
    __slots__ = ("Op", "K", "V")

    def __init__(self, op, k, v):
        self.Op, self.K, self.V = op, k, v


class State:
    def __init__(self):
        self.Store = {}  # map[Key]Value


def Conflict(gamma, delta):  # state.go:53-60
    if gamma.K == delta.K:
        if gamma.Op == PUT or delta.Op == PUT:
            return True
    return False


def ConflictBatch(batch1, batch2):  # state.go:62-71
    for i in range(len(batch1)):
        for j in range(len(batch2)):
            if Conflict(batch1[i], batch2[j]):
                return True
    return False


def IsRead(command):  # state.go:73-75
    return command.Op == GET


def Execute(c, st):  # (*Command).Execute  state.go:77-103
    if c.Op == PUT:
        st.Store[c.K] = c.V  # :93
        return c.V           # :94
    if c.Op == GET:
        if c.K in st.Store:  # :97
            return st.Store[c.K]
    return NIL               # :102


# ---- Go-shaped replica objects ------------------------------------------------------------------
class LeaderBookkeeping:
    """minpaxosproto.LeaderBookkeeping (minpaxosproto.go:17-24) / paxos.LeaderBookkeeping
    (paxos.go:58-65)"""

    def __init__(self, acceptOKs=0, nacks=0, maxRecvBallot=0, prepareOKs=0,
                 clientProposals=None):
        self.AcceptOKs, self.Nacks, self.MaxRecvBallot = acceptOKs, nacks, maxRecvBallot
        self.PrepareOKs, self.ClientProposals = prepareOKs, clientProposals


class Instance:
    def __init__(self, status, ballot=0, cmds=None, lb=None):
        self.Status, self.Ballot, self.Cmds, self.Lb = status, ballot, cmds, lb


class PrepareBookkeeping:  # bareminpaxos.go:64-71
    def __init__(self, N):
        self.prepareOKs = 0
        self.peerCommits = [0] * N
        self.highestInstanceNumber = -1
        self.maxRecvBallot = 0
        self.cmds = None


class Replica:
    """the fields of bareminpaxos.Replica / paxos.Replica the hot path touches, plus an event
    log standing in for the side effects the engine reports as flags (recordInstanceMetadata,
    sync, bcastAccept, ProposeChan, the catch-up copy)"""

    def __init__(self, N, instanceSpace, committedUpTo=-1, defaultBallot=-1):
        self.N = N
        self.instanceSpace = instanceSpace
        self.committedUpTo = committedUpTo
        self.defaultBallot = defaultBallot
        self.prepareBookkeeping = PrepareBookkeeping(N)
        self.State = State()
        self.events = []

    # ---- MIN  src/bareminpaxos/bareminpaxos.go ----
    def min_handleAcceptReply(self, areply):  # :1014-1064
        inst = self.instanceSpace[areply.Instance]                     # :1015
        if areply.OK == TRUE:                                          # :1023
            lb = deref(deref(inst, "inst").Lb, "inst.Lb")
            lb.AcceptOKs = i32(lb.AcceptOKs + 1)                       # :1024
            if lb.AcceptOKs + 1 > i32(self.N) >> 1:                    # :1025
                if lb.AcceptOKs == i32(self.N) >> 1:                   # :1026
                    inst.Status = COMMITTED                            # :1028
                    self.events.append(("commit", areply.Instance))    # :1045-1046
                    self.committedUpTo = areply.Instance               # :1048
                setidx(self.prepareBookkeeping.peerCommits, areply.Id,
                       i32(areply.Instance - 1))                       # :1050

    def min_handlePrepareReply(self, preply):  # :912-966
        if self.defaultBallot > preply.Ballot:                         # :916
            return
        if self.defaultBallot == preply.Ballot:                        # :921
            pb = self.prepareBookkeeping
            pb.prepareOKs = i32(pb.prepareOKs + 1)                     # :922
            setidx(pb.peerCommits, preply.Id, preply.LastCommitted)    # :923
            if preply.Instance > pb.highestInstanceNumber or (
                    preply.Instance == pb.highestInstanceNumber and
                    preply.Ballot > pb.maxRecvBallot):                 # :925
                pb.cmds = preply.Command                               # :927
                pb.maxRecvBallot = preply.Ballot                       # :928
                pb.highestInstanceNumber = preply.Instance             # :930
                self.events.append(("selected",))
            if self.committedUpTo <= preply.LastCommitted:             # :934
                # :936-938 copy CatchUpLog[i-(committedUpTo+1)] into instanceSpace[i]
                self.events.append(("catchup", self.committedUpTo + 1))
                self.committedUpTo = preply.LastCommitted              # :939
            if pb.prepareOKs == i32(self.N) >> 1 and \
                    pb.highestInstanceNumber > self.committedUpTo:     # :945
                # :948-952 instanceSpace[highest] = {defaultBallot, ACCEPTED, lb, cmds}
                self.committedUpTo = pb.highestInstanceNumber          # :954
                self.events.append(("bcastAccept",))                  # :956-958

    def min_executeCommands(self, i):  # :1066-1098, one pass of the outer loop from cursor i
        while i <= self.committedUpTo:                                 # :1071
            inst = self.instanceSpace.get_or_nil(i)
            if inst is None:  # CONTRACT: an instance not yet received stops the cursor
                break
            if inst.Cmds is not None:                                  # :1072
                for j in range(len(inst.Cmds)):                        # :1074
                    val = Execute(inst.Cmds[j], self.State)            # :1075
                    self.events.append(("exec", inst.Cmds[j], val))
                i += 1                                                 # :1086
            else:
                break                                                  # :1089
        return i

    # ---- CLASSIC  src/paxos/paxos.go ----
    def updateCommittedUpTo(self):  # :259-264
        while True:
            nxt = self.instanceSpace.get_or_nil(self.committedUpTo + 1)
            if nxt is not None and nxt.Status == COMMITTED:
                self.committedUpTo += 1
            else:
                break

    def classic_handleAcceptReply(self, areply):  # :631-673
        inst = deref(self.instanceSpace[areply.Instance], "inst")      # :632
        if inst.Status != PREPARED and inst.Status != ACCEPTED:        # :634
            return
        lb = deref(inst.Lb, "inst.lb")
        if areply.OK == TRUE:                                          # :639
            lb.AcceptOKs = i32(lb.AcceptOKs + 1)                       # :640
            if lb.AcceptOKs + 1 > self.N >> 1:                         # :641
                inst = self.instanceSpace[areply.Instance]             # :642
                inst.Status = COMMITTED                                # :643
                self.events.append(("commit", areply.Instance))        # :656-657
                self.updateCommittedUpTo()                             # :659
        else:
            lb.Nacks = i32(lb.Nacks + 1)                               # :665
            if areply.Ballot > lb.MaxRecvBallot:                       # :666
                lb.MaxRecvBallot = areply.Ballot                       # :667

    def classic_handlePrepareReply(self, preply):  # :577-629
        inst = deref(self.instanceSpace[preply.Instance], "inst")      # :578
        if inst.Status != PREPARING:                                   # :580
            return
        lb = deref(inst.Lb, "inst.lb")
        if preply.OK == TRUE:                                          # :586
            lb.PrepareOKs = i32(lb.PrepareOKs + 1)                     # :587
            if preply.Ballot > lb.MaxRecvBallot:                       # :589
                inst.Cmds = preply.Command                             # :590
                lb.MaxRecvBallot = preply.Ballot                       # :591
                if lb.ClientProposals is not None:                     # :592
                    self.events.append(("requeue", preply.Instance))   # :596-598
                    lb.ClientProposals = None                          # :599
            if lb.PrepareOKs + 1 > self.N >> 1:                        # :603
                inst.Status = PREPARED                                 # :604
                lb.Nacks = 0                                           # :605
                if inst.Ballot > self.defaultBallot:                   # :606
                    self.defaultBallot = inst.Ballot                   # :607
                self.events.append(("bcastAccept", preply.Instance))   # :609-611
        else:
            lb.Nacks = i32(lb.Nacks + 1)                               # :615
            if preply.Ballot > lb.MaxRecvBallot:                       # :616
                lb.MaxRecvBallot = preply.Ballot                       # :617
            if lb.Nacks >= self.N >> 1:                                # :619
                if lb.ClientProposals is not None:                     # :620
                    self.events.append(("requeue", preply.Instance))   # :622-624
                    lb.ClientProposals = None                          # :625


# ---- wire structs (the decoded messages the handlers receive) -----------------------------------
class AcceptReply:  # minpaxosproto.AcceptReply {Instance, OK, Ballot, Id} / paxosproto (no Id)
    def __init__(self, r):
        self.Instance, self.OK = int(r["instance"]), int(r["ok"])
        self.Ballot, self.Id = int(r["ballot"]), int(r["id"])


class PrepareReply:  # paxosproto.PrepareReply {Instance, OK, Ballot, Command}
    def __init__(self, r):
        self.Instance, self.OK = int(r["instance"]), int(r["ok"])
        self.Ballot, self.Command = int(r["ballot"]), int(r["value_id"])


class MinPrepareReply:  # minpaxosproto.PrepareReply {Id, Instance, OK, Ballot, LastCommitted, ..}
    def __init__(self, r):
        self.Id, self.Instance, self.OK = int(r["id"]), int(r["instance"]), int(r["ok"])
        self.Ballot, self.LastCommitted = int(r["ballot"]), int(r["last_committed"])
        self.Command = int(r["value_id"])


# ---- adapter: the engine's records <-> the objects above ----------------------------------------
def _check_n(N):
    if N < 1 or N > R.MAX_REPLICAS:
        raise GoPanic(R.E_INVAL, "N")


def _inst_from(s):
    if int(s["status"]) == R.STATUS_NIL:
        return None
    return Instance(int(s["status"]), lb=LeaderBookkeeping(
        int(s["accept_oks"]), int(s["nacks"]), int(s["max_recv_ballot"])))


def _inst_to(inst, s):
    s["status"] = inst.Status
    s["accept_oks"], s["nacks"] = inst.Lb.AcceptOKs, inst.Lb.Nacks
    s["max_recv_ballot"] = inst.Lb.MaxRecvBallot


class GoBackend:
    """the Oracle/Engine call surface over the transliteration (GoPanic where Go panics)"""

    def __init__(self, n_replicas=5, mode=R.MODE_MIN, kv_per_group=512):
        self.N, self.mode, self.K = n_replicas, mode, kv_per_group
        self.state = State()

    def _tally(self, rep, recs):
        h = rep.min_handleAcceptReply if self.mode == R.MODE_MIN else rep.classic_handleAcceptReply
        for r in recs:
            h(AcceptReply(r))

    def accept_tally(self, recs, st, inst_base=0, committed_upto=-1, peer_commits=None,
                     want_decided=True):
        _check_n(self.N)
        st = np.array(st, R.INST_STATE, copy=True)
        space = Slice(inst_base, [_inst_from(s) for s in st])
        rep = Replica(self.N, space, committed_upto)
        if peer_commits is not None:
            rep.prepareBookkeeping.peerCommits = [int(x) for x in peer_commits]
        self._tally(rep, recs)
        dec = np.zeros(len(st), np.uint8)
        for ev in rep.events:
            dec[ev[1] - inst_base] = 1
        for j, inst in enumerate(space.items):
            if inst is not None:
                _inst_to(inst, st[j])
        pc = np.array(rep.prepareBookkeeping.peerCommits, np.int32)
        return st, rep.committedUpTo, pc, dec if want_decided else None

    def committed_prefix(self, st, inst_base, committed_upto):
        rep = Replica(self.N, Slice(inst_base, [_inst_from(s) for s in st]), committed_upto)
        rep.updateCommittedUpTo()
        return rep.committedUpTo

    def prepare_select(self, recs, st, inst_base=0, default_ballot=-1, want_prepared=True):
        _check_n(self.N)
        st = np.array(st, R.PREP_STATE, copy=True)
        items = []
        for s in st:
            if int(s["status"]) == R.STATUS_NIL:
                items.append(None)
                continue
            props = [object()] if int(s["flags"]) & R.PF_HAS_PROPOSALS else None
            items.append(Instance(int(s["status"]), int(s["ballot"]), int(s["value_id"]),
                                  LeaderBookkeeping(nacks=int(s["nacks"]),
                                                    maxRecvBallot=int(s["max_recv_ballot"]),
                                                    prepareOKs=int(s["prepare_oks"]),
                                                    clientProposals=props)))
        space = Slice(inst_base, items)
        rep = Replica(self.N, space, defaultBallot=default_ballot)
        for r in recs:
            rep.classic_handlePrepareReply(PrepareReply(r))
        prep = np.zeros(len(st), np.uint8)
        requeued, bcast = set(), set()
        for ev in rep.events:
            (requeued if ev[0] == "requeue" else bcast).add(ev[1] - inst_base)
        touched = {int(r["instance"]) - inst_base for r in recs}
        for j in touched:
            inst, s = items[j], st[j]
            s["status"], s["ballot"], s["value_id"] = inst.Status, inst.Ballot, inst.Cmds
            s["prepare_oks"], s["nacks"] = inst.Lb.PrepareOKs, inst.Lb.Nacks
            s["max_recv_ballot"] = inst.Lb.MaxRecvBallot
            # CONTRACT: the flags describe this call on every instance that had replies
            fl = int(s["flags"]) & ~(R.PF_HAS_PROPOSALS | R.PF_REQUEUED | R.PF_PREPARED_NOW)
            fl |= R.PF_HAS_PROPOSALS if inst.Lb.ClientProposals is not None else 0
            fl |= R.PF_REQUEUED if j in requeued else 0
            fl |= R.PF_PREPARED_NOW if j in bcast else 0
            s["flags"] = fl
        for j in bcast:
            prep[j] = 1
        return st, rep.defaultBallot, prep if want_prepared else None

    def prepare_select_min(self, recs, grp_rec_off, gst, peer_commits=None, want_effects=True):
        _check_n(self.N)
        N = self.N
        off = [int(x) for x in grp_rec_off]
        gst = np.array(gst, R.GROUP_PREP_STATE, copy=True)
        G = len(gst)
        if off[0] != 0 or off[G] != len(recs) or any(off[g + 1] < off[g] for g in range(G)):
            raise GoPanic(R.E_INVAL, "offsets")
        pc = np.zeros(G * N, np.int32) if peer_commits is None else \
            np.array(peer_commits, np.int32, copy=True).reshape(-1)
        eff = np.zeros(len(recs), R.PREPARE_EFFECT)
        for g in range(G):
            s = gst[g]
            rep = Replica(N, None, int(s["committed_upto"]), int(s["default_ballot"]))
            pb = rep.prepareBookkeeping
            pb.prepareOKs, pb.maxRecvBallot = int(s["prepare_oks"]), int(s["max_recv_ballot"])
            pb.highestInstanceNumber, pb.cmds = int(s["highest_instance"]), int(s["value_id"])
            pb.peerCommits = [int(x) for x in pc[g * N:(g + 1) * N]]
            triggered = int(s["triggered"])
            for p in range(off[g], off[g + 1]):
                pr = MinPrepareReply(recs[p])
                counted = rep.defaultBallot == pr.Ballot
                rep.events = []
                rep.min_handlePrepareReply(pr)
                fl, frm = (R.EF_COUNTED if counted else 0), -1
                for ev in rep.events:
                    if ev[0] == "selected":
                        fl |= R.EF_SELECTED
                    elif ev[0] == "catchup":
                        fl |= R.EF_CATCHUP
                        frm = ev[1]
                    else:
                        fl |= R.EF_TRIGGER
                        triggered += 1
                eff[p]["flags"], eff[p]["catchup_from"] = fl, frm
            s["prepare_oks"], s["max_recv_ballot"] = pb.prepareOKs, pb.maxRecvBallot
            s["highest_instance"], s["value_id"] = pb.highestInstanceNumber, pb.cmds
            s["committed_upto"], s["triggered"] = rep.committedUpTo, triggered
            pc[g * N:(g + 1) * N] = pb.peerCommits
        return gst, pc, eff if want_effects else None

    # executeCommands' inner loop over one log slice (bareminpaxos.go:1074-1075) and the
    # Conflict of each command with the previous command on its key in the slice
    def apply(self, op, key, val, want_conf=True):
        m = len(op)
        ret = np.zeros(m, np.int64)
        conf = np.zeros(m, np.uint8)
        last = {}
        for i in range(m):
            c = Command(int(op[i]), int(key[i]), int(val[i]))
            if c.K in last:
                conf[i] = Conflict(last[c.K], c)
            last[c.K] = c
            ret[i] = Execute(c, self.state)
        return ret, conf if want_conf else None

    def kv_export(self):
        items = sorted(self.state.Store.items())
        return (np.array([k for k, _ in items], np.int64),
                np.array([v for _, v in items], np.int64))

    def conflict_batch(self, op, key, inst_off):
        off = [int(x) for x in inst_off]
        cmds = [Command(int(op[i]), int(key[i]), 0) for i in range(len(op))]
        out = [ConflictBatch(cmds[off[i]:off[i + 1]], cmds[off[i + 1]:off[i + 2]])
               for i in range(len(off) - 2)]
        return np.array(out, np.uint8)

    # ---- fused group step: a batch of handleAcceptReply, then executeCommands, per group ----
    def group_step(self, b, kv_cnt=None, kv_key=None, kv_val=None, want_conf=True,
                   want_decided=True):
        _check_n(self.N)
        G, ipg, N, K = int(b["n_groups"]), int(b["ipg"]), self.N, self.K
        recs, roff = b["recs"], [int(x) for x in b["grp_rec_off"]]
        st_in = np.asarray(b["st_in"], R.INST_STATE)
        coff = [int(x) for x in b["cmd_off"]]
        has = b.get("has_cmds")
        op, key, val = b["op"], b["key"], b["val"]
        m = len(op)
        kci = np.zeros(G, np.uint32) if kv_cnt is None else np.asarray(kv_cnt, np.uint32)
        kko = np.zeros(G * K, np.int64) if kv_key is None else np.array(kv_key, np.int64)
        kvo = np.zeros(G * K, np.int64) if kv_val is None else np.array(kv_val, np.int64)
        out = dict(st_out=st_in.copy(), committed_out=np.zeros(G, np.int32),
                   executed_out=np.zeros(G, np.int32), peer_out=np.zeros(G * N, np.int32),
                   ret=np.zeros(m, np.int64), conf_prev=np.zeros(m, np.uint8),
                   kv_cnt=np.zeros(G, np.uint32), kv_key=kko, kv_val=kvo,
                   decided=np.zeros(G * ipg, np.uint8), n_decided=np.zeros(G, np.uint32))
        for g in range(G):
            # handleAcceptReply over the group's replies
            space = Slice(0, [_inst_from(s) for s in st_in[g * ipg:(g + 1) * ipg]])
            rep = Replica(N, space, int(b["committed_in"][g]))
            rep.prepareBookkeeping.peerCommits = [int(x) for x in b["peer_in"][g * N:(g + 1) * N]]
            self._tally(rep, recs[roff[g]:roff[g + 1]])
            for ev in rep.events:
                out["decided"][g * ipg + ev[1]] = 1
            out["n_decided"][g] = int(out["decided"][g * ipg:(g + 1) * ipg].sum())
            for i in {int(r["instance"]) for r in recs[roff[g]:roff[g + 1]]}:
                _inst_to(space[i], out["st_out"][g * ipg + i])
            out["committed_out"][g] = rep.committedUpTo
            out["peer_out"][g * N:(g + 1) * N] = rep.prepareBookkeeping.peerCommits
            # the instances' command slices (Cmds == nil where has_cmds says so)
            cmd_index = {}
            for i, inst in enumerate(space.items):
                if inst is None:
                    continue
                gi = g * ipg + i
                if has is not None and not has[gi]:
                    continue
                inst.Cmds = [Command(int(op[c]), int(key[c]), int(val[c]))
                             for c in range(coff[gi], coff[gi + 1])]
                for j, c in enumerate(range(coff[gi], coff[gi + 1])):
                    cmd_index[id(inst.Cmds[j])] = c
            # CONTRACT: the group's table in order; a Go map keeps no order, this one keeps
            # insertion order, which is the table layout (existing slots, then first PUTs)
            cnt = int(kci[g])
            if cnt > K:
                raise GoPanic(R.E_INVAL, "kv_cnt")
            for e in range(cnt):
                rep.State.Store[int(kko[g * K + e])] = int(kvo[g * K + e])
            rep.events = []
            ex = rep.min_executeCommands(int(b["executed_in"][g]) + 1) - 1
            last = {}
            for ev in rep.events:
                _, c, v = ev
                at = cmd_index[id(c)]
                out["conf_prev"][at] = Conflict(last[c.K], c) if c.K in last else 0
                last[c.K] = c
                out["ret"][at] = v
            out["executed_out"][g] = ex
            if len(rep.State.Store) > K:
                raise GoPanic(R.E_KV_FULL, "group table full")
            out["kv_cnt"][g] = len(rep.State.Store)
            for e, (k, v) in enumerate(rep.State.Store.items()):
                kko[g * K + e], kvo[g * K + e] = k, v
        if not want_conf:
            out["conf_prev"] = None
        if not want_decided:
            out["decided"] = None
        return out
