// oracle/wire.cpp — TEST INFRASTRUCTURE ONLY. CPU restatement of the peer-stream framing
// (SURVEY §8(f) rank 1); the parity checker for minpaxos_amd/csrc/decode.hip.
//
// genericsmr.(*Replica).replicaListener  src/genericsmr/genericsmr.go:402-446, one frame per
// loop iteration: ReadByte() the code (:410), then
//   GENERIC_SMR_BEACON / _REPLY (6, 7): Beacon/BeaconReply.Unmarshal, 8 bytes (:414-428)
//   rpcTable codes (:433-439), registered 8..13 by bareminpaxos.NewReplica (:108-113):
//     Prepare.Unmarshal          ReadAtLeast 12   minpaxosprotomarsh.go:259-270
//     Accept / Commit / PrepareReply: varint-prefixed slices (:470-507, :648-672, :352-387)
//     CommitShort.Unmarshal      ReadAtLeast 16   :737-749
//     AcceptReply.Unmarshal      13 bytes, LE     :568-580 (written by Marshal :545-566)
//   anything else: log "unknown message type" and continue with the next byte (:440-442).
// The engine's contract stops at variable-length frames and at a frame that runs past the end
// of the buffer (include/mpx.h, mpx_decode_peer_stream); this restatement does the same.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/mpx.h"

namespace {

int32_t le32(const uint8_t* b) {
    return (int32_t)((uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) |
                     ((uint32_t)b[3] << 24));
}

// body length after the code byte; -1 = variable-length message
int body_len(uint8_t code) {
    switch (code) {
    case MPX_PEER_BEACON:
    case MPX_PEER_BEACON_REPLY: return 8;
    case MPX_PEER_PREPARE: return 12;
    case MPX_PEER_COMMIT_SHORT: return 16;
    case MPX_PEER_ACCEPT_REPLY: return 13;
    case MPX_PEER_ACCEPT:
    case MPX_PEER_COMMIT:
    case MPX_PEER_PREPARE_REPLY: return -1;
    default: return 0;  // unknown code: only the code byte is consumed
    }
}

}  // namespace

extern "C" {

int orc_decode_peer_stream(const uint8_t* buf, size_t len, mpx_accept_reply* ar, size_t ar_cap,
                           mpx_peer_frame* other, size_t other_cap, mpx_decode_result* res) {
    size_t p = 0;
    uint64_t n_ar = 0, n_oth = 0;
    int32_t why = MPX_DECODE_END, code_at = -1;
    while (p < len) {
        const uint8_t code = buf[p];
        const int bl = body_len(code);
        if (bl < 0) {
            why = MPX_DECODE_VARIABLE;
            code_at = code;
            break;
        }
        if (p + 1 + (size_t)bl > len) {
            why = MPX_DECODE_PARTIAL;
            code_at = code;
            break;
        }
        if (code == MPX_PEER_ACCEPT_REPLY) {
            const uint8_t* b = buf + p + 1;
            if (n_ar < ar_cap) {
                mpx_accept_reply r;
                memset(&r, 0, sizeof(r));
                r.instance = le32(b);      // t.Instance  bs[0:4]
                r.ok = b[4];               // t.OK        bs[4]
                r.ballot = le32(b + 5);    // t.Ballot    bs[5:9]
                r.id = le32(b + 9);        // t.Id        bs[9:13]
                ar[n_ar] = r;
            }
            ++n_ar;
        } else {
            if (n_oth < other_cap) {
                mpx_peer_frame f;
                memset(&f, 0, sizeof(f));
                f.offset = (uint32_t)p;
                f.code = code;
                other[n_oth] = f;
            }
            ++n_oth;
        }
        p += 1 + (size_t)bl;
    }
    res->consumed = p;
    res->n_accept_replies = n_ar;
    res->n_other = n_oth;
    res->stop_reason = why;
    res->stop_code = code_at;
    return MPX_OK;
}

// Full peer-stream framing (mpx_decode_stream): replicaListener (genericsmr.go:402-446) with the
// rpcTable of bareminpaxos (MIN, bareminpaxos.go:108-113) or paxos (CLASSIC, paxos.go:93-98),
// every message Unmarshal()ed as its Go code reads it:
//   binary.ReadVarint = ReadUvarint (10 bytes at most; a 10th byte > 1 overflows) + zig-zag;
//   a negative slice length makes make() panic; a Command / Instance / header whose bytes are
//   not all in the buffer yet is a partial frame (on the socket, Unmarshal would block).
namespace {

enum VarStatus { kVarOk = 0, kVarPartial = 1, kVarMalformed = 2 };

// binary.ReadVarint at *pos; advances *pos
int read_varint(const uint8_t* buf, size_t len, size_t* pos, int64_t* out) {
    uint64_t x = 0;
    unsigned s = 0;
    for (int i = 0; i < 10; ++i) {
        if (*pos >= len) return kVarPartial;
        const uint8_t b = buf[(*pos)++];
        if (b < 0x80) {
            if (i == 9 && b > 1) return kVarMalformed;  // errOverflow
            x |= (uint64_t)b << s;
            *out = (int64_t)(x >> 1) ^ -(int64_t)(x & 1);  // zig-zag: ux>>1, ^ if ux&1
            return kVarOk;
        }
        x |= (uint64_t)(b & 0x7f) << s;
        s += 7;
    }
    return kVarMalformed;
}

// a slice of n 17-byte Commands at *pos (make([]state.Command, n) + n Command.Unmarshal)
int skip_cmds(size_t len, size_t* pos, int64_t n) {
    if (n < 0) return kVarMalformed;  // makeslice: len out of range
    if ((uint64_t)n > (len - *pos) / 17) return kVarPartial;
    *pos += 17 * (size_t)n;
    return kVarOk;
}

// body of a variable-length message at p (code byte at p); fills f
int parse_var(int proto, const uint8_t* buf, size_t len, size_t p, mpx_var_frame* f) {
    const uint8_t code = buf[p];
    size_t hdr;
    bool log = false;
    if (proto == MPX_MODE_MIN) {
        hdr = code == MPX_PEER_ACCEPT ? 16 : code == MPX_PEER_COMMIT ? 12 : 17;
        log = code != MPX_PEER_COMMIT;  // Accept and PrepareReply carry a CatchUpLog
    } else {
        hdr = code == MPX_PEER_PREPARE_REPLY ? 9 : 12;
    }
    memset(f, 0, sizeof(*f));
    f->offset = (uint32_t)p;
    f->code = code;
    size_t pos = p + 1 + hdr;
    if (pos > len) return kVarPartial;  // ReadAtLeast(header)
    int64_t n = 0;
    int st = read_varint(buf, len, &pos, &n);
    if (st) return st;
    if (n < 0) return kVarMalformed;
    f->cmds_off = (uint32_t)pos;
    if ((st = skip_cmds(len, &pos, n))) return st;
    f->n_cmds = (uint32_t)n;
    f->log_off = (uint32_t)pos;
    if (log) {
        int64_t m = 0;
        if ((st = read_varint(buf, len, &pos, &m))) return st;
        if (m < 0) return kVarMalformed;
        if ((uint64_t)m > (len - pos) / 9) return kVarPartial;  // >= 9 bytes per Instance
        f->log_off = (uint32_t)pos;
        for (int64_t i = 0; i < m; ++i) {  // Instance.Unmarshal: Ballot, Status, Cmds
            if (pos + 8 > len) return kVarPartial;
            pos += 8;
            int64_t k = 0;
            if ((st = read_varint(buf, len, &pos, &k))) return st;
            if ((st = skip_cmds(len, &pos, k))) return st;
        }
        f->n_log = (uint32_t)m;
    }
    f->length = (uint32_t)(pos - p);
    return kVarOk;
}

// fixed body length (0 = unknown code, 1-byte frame), or -1 = variable-length message
int fixed_body(int proto, uint8_t code) {
    switch (code) {
    case MPX_PEER_BEACON:
    case MPX_PEER_BEACON_REPLY: return 8;
    case MPX_PEER_PREPARE: return proto == MPX_MODE_MIN ? 12 : 13;
    case MPX_PEER_COMMIT_SHORT: return 16;
    case MPX_PEER_ACCEPT_REPLY: return proto == MPX_MODE_MIN ? 13 : 9;
    case MPX_PEER_ACCEPT:
    case MPX_PEER_COMMIT:
    case MPX_PEER_PREPARE_REPLY: return -1;
    default: return 0;
    }
}

}  // namespace

int orc_decode_stream(int proto, const uint8_t* buf, size_t len, const mpx_decode_out* out,
                      mpx_stream_result* res) {
    if (proto != MPX_MODE_MIN && proto != MPX_MODE_CLASSIC) return MPX_E_INVAL;
    size_t p = 0;
    uint64_t n_ar = 0, n_prep = 0, n_var = 0, n_oth = 0;
    int32_t why = MPX_DECODE_END, code_at = -1;
    while (p < len) {
        const uint8_t code = buf[p];
        const int bl = fixed_body(proto, code);
        const uint8_t* b = buf + p + 1;
        if (bl < 0) {
            mpx_var_frame f;
            const int st = parse_var(proto, buf, len, p, &f);
            if (st) {
                why = st == kVarPartial ? MPX_DECODE_PARTIAL : MPX_DECODE_MALFORMED;
                code_at = code;
                break;
            }
            if (code == MPX_PEER_PREPARE_REPLY) {
                if (n_prep < out->prep_cap) {
                    if (proto == MPX_MODE_MIN) {  // Id, Instance, OK, Ballot, LastCommitted
                        mpx_prepare_reply_min r;
                        r.id = le32(b);
                        r.instance = le32(b + 4);
                        r.ok = b[8];
                        r.ballot = le32(b + 9);
                        r.last_committed = le32(b + 13);
                        r.value_id = (uint32_t)n_var;
                        ((mpx_prepare_reply_min*)out->prep)[n_prep] = r;
                    } else {  // Instance, OK, Ballot
                        mpx_prepare_reply r;
                        r.instance = le32(b);
                        r.ok = b[4];
                        r.ballot = le32(b + 5);
                        r.value_id = (uint32_t)n_var;
                        ((mpx_prepare_reply*)out->prep)[n_prep] = r;
                    }
                }
                ++n_prep;
            }
            if (n_var < out->var_cap) out->var[n_var] = f;
            ++n_var;
            p += f.length;
            continue;
        }
        if (p + 1 + (size_t)bl > len) {
            why = MPX_DECODE_PARTIAL;
            code_at = code;
            break;
        }
        if (code == MPX_PEER_ACCEPT_REPLY) {
            if (n_ar < out->ar_cap) {
                mpx_accept_reply r;
                memset(&r, 0, sizeof(r));
                r.instance = le32(b);  // Instance, OK, Ballot (+ Id for MIN)
                r.ok = b[4];
                r.ballot = le32(b + 5);
                r.id = proto == MPX_MODE_MIN ? le32(b + 9) : -1;
                out->ar[n_ar] = r;
            }
            ++n_ar;
        } else {
            if (n_oth < out->other_cap) {
                mpx_peer_frame f;
                memset(&f, 0, sizeof(f));
                f.offset = (uint32_t)p;
                f.code = code;
                out->other[n_oth] = f;
            }
            ++n_oth;
        }
        p += 1 + (size_t)bl;
    }
    res->consumed = p;
    res->next = p;
    res->n_accept_replies = n_ar;
    res->n_prepare_replies = n_prep;
    res->n_var = n_var;
    res->n_other = n_oth;
    res->stop_reason = why;
    res->stop_code = code_at;
    return MPX_OK;
}

// Client reply fan-out: every reply, in execution order, is one
// genericsmr.(*Replica).ReplyProposeTS(reply, client writer) (genericsmr.go:529-535), i.e.
// ProposeReplyTS.Marshal (gsmrprotomarsh.go:702-732) appended to that client's stream:
// OK u8, CommandId i32, Value i64 (state.Value.Marshal, statemarsh.go:48-53), Timestamp i64,
// Leader i32, little endian. out holds the clients' streams back to back, client 0 first.
int orc_encode_replies(const mpx_reply_rec* recs, size_t n, uint32_t n_clients, uint8_t ok,
                       int32_t leader, uint8_t* out, uint64_t* client_off) {
    if (!n_clients) return MPX_E_INVAL;
    std::vector<std::vector<uint8_t>> wire(n_clients);
    for (size_t i = 0; i < n; ++i) {
        const mpx_reply_rec& r = recs[i];
        if (r.client >= n_clients) return MPX_E_INVAL;
        std::vector<uint8_t>& w = wire[r.client];
        w.push_back(ok);
        for (int k = 0; k < 4; ++k) w.push_back((uint8_t)((uint32_t)r.command_id >> (8 * k)));
        for (int k = 0; k < 8; ++k) w.push_back((uint8_t)((uint64_t)r.value >> (8 * k)));
        for (int k = 0; k < 8; ++k) w.push_back((uint8_t)((uint64_t)r.timestamp >> (8 * k)));
        for (int k = 0; k < 4; ++k) w.push_back((uint8_t)((uint32_t)leader >> (8 * k)));
    }
    uint64_t o = 0;
    for (uint32_t c = 0; c < n_clients; ++c) {
        client_off[c] = o;
        if (!wire[c].empty()) memcpy(out + o, wire[c].data(), wire[c].size());
        o += wire[c].size();
    }
    client_off[n_clients] = o;
    return MPX_OK;
}

// Instance-log encodings of a run of log records:
//   MPX_LOG_CATCHUP  (*Instance).Marshal  minpaxosprotomarsh.go:100-124: Ballot (4 bytes LE),
//                    int32(Status) (4), binary.PutVarint(len(Cmds)) written as b[0:wlen] (:117-120),
//                    then Cmds[i].Marshal (statemarsh.go:8-19): Op byte, K and V little endian.
//   MPX_LOG_DURABLE  recordInstanceMetadata  bareminpaxos.go:164-174 (Ballot, Status, instNo as
//                    LittleEndian.PutUint32) + recordCommands :177-188 (nil -> nothing).
namespace {
size_t put_varint(uint8_t* b, int64_t x) {  // encoding/binary.PutVarint
    uint64_t ux = (uint64_t)x << 1;
    if (x < 0) ux = ~ux;
    size_t i = 0;
    while (ux >= 0x80) {
        b[i++] = (uint8_t)(ux | 0x80);
        ux >>= 7;
    }
    b[i++] = (uint8_t)ux;
    return i;
}
void put_le(std::vector<uint8_t>& w, uint64_t v, int bytes) {
    for (int k = 0; k < bytes; ++k) w.push_back((uint8_t)(v >> (8 * k)));
}
}  // namespace

int orc_encode_log(int format, const mpx_log_rec* recs, size_t n, const uint64_t* cmd_off,
                   const uint8_t* op, const int64_t* key, const int64_t* val, uint8_t* out,
                   size_t out_cap, uint64_t* rec_off) {
    if (format != MPX_LOG_CATCHUP && format != MPX_LOG_DURABLE) return MPX_E_INVAL;
    std::vector<uint8_t> w;
    for (size_t i = 0; i < n; ++i) {
        rec_off[i] = w.size();
        const mpx_log_rec& r = recs[i];
        const uint64_t c0 = cmd_off[i], c1 = cmd_off[i + 1];
        put_le(w, (uint32_t)r.ballot, 4);
        put_le(w, (uint32_t)r.status, 4);
        if (format == MPX_LOG_CATCHUP) {
            uint8_t b[10];
            const size_t l = put_varint(b, (int64_t)(c1 - c0));
            w.insert(w.end(), b, b + l);
        } else {
            put_le(w, (uint32_t)r.inst_no, 4);
        }
        for (uint64_t j = c0; j < c1; ++j) {
            w.push_back(op[j]);
            put_le(w, (uint64_t)key[j], 8);
            put_le(w, (uint64_t)val[j], 8);
        }
    }
    rec_off[n] = w.size();
    if (w.size() > out_cap) return MPX_E_INVAL;
    if (!w.empty()) memcpy(out, w.data(), w.size());
    return MPX_OK;
}

// Durable-log replay: bareminpaxos.(*Replica).getDataFromStableStore bareminpaxos.go:122-161,
// one record per loop iteration, in file order: 12 metadata bytes (:127-140), one
// Command.Unmarshal (:142-143, statemarsh.go:21-37), the two watermark updates (:145-151), and
// instanceSpace[instNo] = the record (:153-157; last_rec[] keeps the index of that record).
// A trailing partial record is rejected (the reference decodes it zero-padded), and an instNo
// outside [0, inst_cap) stops the loop where Go's index check panics. Record i of this call is
// file record rec_base + i (a store replayed in chunks); last_rec is in/out.
int orc_replay_durable(const uint8_t* log, size_t len, int32_t inst_cap, int32_t rec_base,
                       mpx_log_rec* recs, uint8_t* op, int64_t* key, int64_t* val,
                       int32_t* last_rec, int32_t* scalars) {
    if (len % MPX_DURABLE_REC_BYTES || rec_base < 0) return MPX_E_INVAL;
    auto u32 = [](const uint8_t* b) {
        return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) |
               ((uint32_t)b[3] << 24);
    };
    auto u64 = [&](const uint8_t* b) { return (uint64_t)u32(b) | ((uint64_t)u32(b + 4) << 32); };
    int32_t& defaultBallot = scalars[0];
    int32_t& committedUpTo = scalars[1];
    const size_t n = len / MPX_DURABLE_REC_BYTES;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* bs = log + i * MPX_DURABLE_REC_BYTES;
        const int32_t ballot = (int32_t)u32(bs);
        const int32_t status = (int32_t)u32(bs + 4);
        const int32_t instNo = (int32_t)u32(bs + 8);
        recs[i] = mpx_log_rec{ballot, status, instNo, 0};
        op[i] = bs[12];
        key[i] = (int64_t)u64(bs + 13);
        val[i] = (int64_t)u64(bs + 21);
        if (ballot > defaultBallot) defaultBallot = ballot;
        if (instNo > committedUpTo && status == MPX_COMMITTED) committedUpTo = instNo;
        if (instNo < 0 || instNo >= inst_cap) return MPX_E_NIL_INSTANCE;
        last_rec[instNo] = rec_base + (int32_t)i;
    }
    return MPX_OK;
}

}  // extern "C"
