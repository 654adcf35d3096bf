// siddhi-hip: compiled NFA program (host-built, device-resident, POD).
//
// The program is the flattened processor graph that the reference builds in
// StateInputStreamParser.parse (core/util/parser/StateInputStreamParser.java:148-408)
// plus the condition trees of its FilterProcessors, lowered to a predicate bytecode.
#pragma once
#include <stdint.h>

#ifndef SHP_HD
#if defined(__HIPCC__)
#define SHP_HD __host__ __device__
#else
#define SHP_HD
#endif
#endif

namespace shp {

constexpr int MAXS = 8;       // states (StateEvent slots)
constexpr int MAXP = 8;       // pre/post processors
constexpr int MAXQ = 4;       // schedulers (absent processors)
constexpr int MAXCOL = 8;     // predicate input columns
constexpr int MAXSTREAM = 8;  // input streams
constexpr int NV = 4;         // attribute values captured per StreamEvent node
constexpr int MAXCODE = 192;  // bytecode instructions
constexpr int MAXSTACK = 12;  // predicate VM stack depth

enum Kind : int8_t { K_STREAM = 0, K_COUNT, K_LOGICAL, K_ABSENT_STREAM, K_ABSENT_LOGICAL };
enum SeqType : int8_t { PATTERN = 0, SEQUENCE = 1 };
enum LType : int8_t { L_AND = 0, L_OR = 1 };
enum Tag : int8_t { T_NULL = 0, T_INT, T_LONG, T_FLOAT, T_DOUBLE, T_BOOL, T_STR };

enum Op : uint8_t {
  OP_END = 0,
  OP_CONST,        // push imm, tag a
  OP_VAR,          // a=state, b=(int8)index, c=column
  OP_ISNULLSTATE,  // a=state, b=(int8)index
  OP_AND,          // short-circuit: pop x; if !TRUE push FALSE, jump d
  OP_ANDEND,       // pop y; push y==TRUE
  OP_OR,           // pop x; if TRUE push TRUE, jump d
  OP_OREND,        // pop y; push y==TRUE
  OP_NOT,          // pop x; push !(x==TRUE)
  OP_ISNULL,       // pop x; push x==NULL
  OP_CMP,          // a=cmp(0 gt 1 ge 2 lt 3 le 4 eq 5 ne), b=promoted tag
  OP_ARITH,        // a=op(0 add 1 sub 2 mul 3 div 4 mod), b=result tag
  OP_IFTE,         // pop else, then, cond; push cond==TRUE ? then : else (ifThenElse)
  OP_COALESCE,     // a=n: pop n values; push the first non-null in argument order (coalesce)
  OP_INSTOF,       // a=tag: pop x; push x's tag == a (instanceOf*; null -> FALSE)
};

struct Instr {
  uint8_t op, a, b, c;
  int32_t d;
  int64_t imm;
};

struct DPre {
  int8_t kind, stateId, isStart, stream;
  int8_t logical, sched, pad0, pad1;
  int16_t withinEvery, thisPost, thisLast, partner, countPost, filterPc;
  int32_t minCount, maxCount;
  int64_t waiting;
};

struct DPost {
  int8_t kind, stateId, hasNext, logical;
  int16_t nextState, nextEvery, thisPre, callbackPre, partnerPre, partnerPost;
  int32_t minCount, maxCount;
};

struct DevProg {
  int32_t type, nstates, npre, nsched, nstream, ncol, ncode;
  int32_t playback, partitioned;
  int64_t within;
  int8_t startIds[MAXS];
  int32_t nstart;
  DPre pre[MAXP];
  DPost post[MAXP];
  int8_t expireOrder[MAXP];
  int8_t initOrder[MAXP];
  int8_t resetOrder[MAXP];
  int8_t updateOrder[MAXP];
  int8_t nexpire, ninit, nreset, nupdate;
  int8_t startup[MAXQ];
  int8_t schedPre[MAXQ];
  int8_t nstartup, pad2, pad3, pad4;
  int8_t recvCount[MAXSTREAM];
  int8_t recvMulti[MAXSTREAM];
  int8_t recvSelector[MAXSTREAM];
  int8_t recvPre[MAXSTREAM][MAXP];
  int8_t colStream[MAXCOL];
  int8_t colTag[MAXCOL];
  int8_t colPos[MAXCOL];
  int8_t streamNcol[MAXSTREAM];
  int8_t streamCols[MAXSTREAM][NV];
  // select-side aggregate folded at emission (SHP_LAYOUT_AGG on the general lanes): 0 none, 1 avg,
  // 2 sum, 3 count, 4 min, 5 max, over the value of state aggState (first event of its chain: the
  // selector's default index 0) in predicate column aggCol
  int8_t aggFn, aggState, aggCol, pad5;
  Instr code[MAXCODE];
};

// Register-only predicate for the specialised kernel: up to two comparisons joined by
// AND/OR, each operand a constant or an attribute of slot 0 (candidate e1) / slot 1 (e2).
struct FOperand {
  int8_t kind;   // 0 const, 1 var
  int8_t state;  // 0 or 1
  int8_t pos;    // value position within the event's predicate columns (0/1)
  int8_t tag;    // value tag
  int32_t pad;
  int64_t imm;
};
struct FTerm {
  int8_t cmp, ptype, pad[6];
  FOperand a, b;
};
struct FPred {
  int32_t n;        // 0: no filter (always true), 1 or 2 terms
  int32_t combine;  // 0 AND, 1 OR
  FTerm t[2];
};

// Recognised shape for the specialised kernel (2-state `every e1=S[f1] -> e2=S[f2] within W`,
// same stream, both states plain stream states, filters expressible as FPred).
struct FastShape {
  int32_t ok;
  int32_t stream;
  int64_t within;
  FPred f1, f2;
};

// Recognised shape for the count-sequence kernel (cseq.h): the sequence
// `every e1=S[f1]<1:M>, e2=S[f2]`, same stream, no `within`, f1 over e1's own value and f2 over
// e2's value and e1[last]'s (FPred operands: state 0 = e1[last], state 1 = e2).
constexpr int CSEQ_MAXM = 8;
struct CseqShape {
  int32_t ok;
  int32_t M;      // max count (1..CSEQ_MAXM)
  int32_t every;  // `every e1=...` (else the start state is armed once)
  int32_t minc;   // min count of e1's <min:M> (1..M)
  FPred f1, f2;
};

// Recognised shape for the logical-absent kernel (labs.h): the playback pattern
// `every (x=X[fx] and y=Y[fy]) -> not Z[fz] for T [within W]` over three distinct streams, each
// read through at most one predicate column; fx reads x, fy reads y, fz reads the Z event, x and y.
struct LaOperand {
  int8_t kind;   // 0 const, 1 var
  int8_t state;  // var: state id
  int8_t tag;    // value tag
  int8_t pad;
  int32_t col;   // var: program column
  int64_t imm;
};
struct LaTermS {
  int8_t cmp, ptype, pad[6];
  LaOperand a, b;
};
struct LaPredS {
  int32_t n, combine;
  LaTermS t[2];
};
struct LabsShape {
  int32_t ok;
  int32_t sx, sy, sz;          // state ids of x, y and the absent state
  int32_t stx, sty, stz;       // their streams
  int32_t colx, coly, colz;    // their predicate column (-1: none)
  int64_t wait, within;        // T, W (-1: no within)
  LaPredS fx, fy, fz;
};

}  // namespace shp
