/*
 * siddhi_hip_ir.h -- the program blob sdh_engine_create takes (include/siddhi_hip.h).
 *
 * The blob is the serialized form of the processor graph the reference's parser builds for a state
 * stream (modules/siddhi-core/src/main/java/org/wso2/siddhi/core/util/parser/
 * StateInputStreamParser.java:77-398, reached from InputStreamParser.java:94-99): one pre/post
 * state-processor pair per state id with their next / next-every / within-every / partner /
 * callback links, each stream's receiver with its processors in registration order, the runtime
 * tree that drives init / reset / update, and the filters and selector outputs as typed postfix
 * bytecode. A JNI host produces it from the StateInputStream its parser already holds; the Python
 * producer is siddhi_amd/planner.py + siddhi_amd/ir.py (ProgramIR.serialize), and
 * tests/native/c1_abi.c builds one by hand from this header alone.
 *
 * Layout: the 8 bytes "SDHIR001", then little-endian int64 words:
 *
 *   program   := SDH_IR_VERSION
 *                n_streams  { n_attrs attr_type* }                    (SDH_T_*, sdh_batch's columns)
 *                n_strings  { n_bytes  ceil(n_bytes / 8) words of UTF-8, zero-padded }
 *                n_queries  { query }
 *                n_partitions { n_keys { stream_idx code } n_query_idx query_idx* }
 *                then, per partition: n_fanout { stream_idx java_hash_of_stream_id id_utf16_len }
 *   query     := query_type within_ms n_states partition_idx selector_present
 *                state * n_states                                     (indexed by state id)
 *                n_start start_state_id*
 *                n_receivers { stream_idx receiver_kind n_procs proc_state_id* }
 *                n_nodes node*                                        (node 0 is the root)
 *                n_outputs code*                                      (the selector's expressions)
 *   state     := kind stream_idx is_start min max logical_type partner next_pre next_every_pre
 *                within_every_pre callback_pre this_last_post has_selector waiting_ms
 *                n_filters code*
 *   node      := node_type a b pre
 *   code      := n_insn insn*
 *   insn      := w0 a b imm           w0 = op | ltype << 8 | rtype << 16 | restype << 24
 *
 * Field meanings (state ids index the query's states; -1 = none):
 *   within_ms       the query's `within` in ms, -1 without one
 *   partition_idx   the partition the query belongs to, -1 for none
 *   kind / min, max a stream state; a count state `<min:max>` (max -1: unbounded); a logical state
 *                   (logical_type SDH_L_AND / SDH_L_OR, partner = the other side's state id); an
 *                   absent state (`not S[..] for waiting_ms`; -2: an absent logical side without `for`)
 *   next_pre        the pre-processor this state's post-processor feeds (StreamPostStateProcessor
 *                   .nextStatePreProcessor); next_every_pre: `every` re-arm target
 *                   (nextEveryStatePreProcessor); within_every_pre: the state whose `within` window
 *                   scopes an `every` (withinEveryPreStateProcessor); callback_pre: a count state's
 *                   callback (CountPreStateProcessor.setCallbackPreStateProcessor)
 *   this_last_post  the post-processor of the last state of this state's inner runtime
 *   has_selector    1: completing this state delivers a match to the selector
 *   receivers       per stream the processors that receive its events, in registration order
 *                   (SDH_R_SINGLE: SingleProcessStreamReceiver, SDH_R_MULTI: MultiProcessStreamReceiver)
 *   node            runtime tree: SDH_N_STREAM (pre = its state), SDH_N_NEXT (a -> b),
 *                   SDH_N_EVERY (a = the inner node), SDH_N_LOGICAL (a, b), SDH_N_COUNT (a)
 *   partition key   code evaluated on the keyed stream's event: its value is the key
 *                   (ValuePartitionExecutor.execute)
 *   fan-out         streams the partition's queries read but no key covers (every event reaches every
 *                   key's clone, PartitionStreamReceiver.java:277-281): String.hashCode and UTF-16
 *                   length of the stream id, which fix the junction-map order
 *
 * Bytecode (a stack machine; Java's typed semantics):
 *   SDH_OP_CONST          push imm as restype: int / long raw, float / double IEEE bits in the low
 *                         32 / 64 bits, bool 0/1, string: the dictionary id of program string imm
 *                         (ProgramIR strings; the host maps them to the ids its batches carry)
 *   SDH_OP_ATTR           push attribute imm (of restype) of the event at chain index b of state a's
 *                         slot (the current event's own state for its filter): b >= 0 the b-th event
 *                         of a count chain, SDH_IDX_CURRENT (-1) its last, SDH_IDX_LAST (-2) the one
 *                         before (StateEvent.getStreamEvent, StateEvent.java:138-182); null when absent
 *   SDH_OP_STREAM_IS_NULL push (state a's slot at chain index b is empty)
 *   SDH_OP_IS_NULL        pop x, push (x is null)
 *   SDH_OP_NOT            pop x, push !(x == true)            (NotConditionExpressionExecutor)
 *   SDH_OP_AND, SDH_OP_OR pop r, l; null counts as false
 *   SDH_OP_CMP            pop r, l; push l (imm = SDH_CMP_*) r, compared in the domain of
 *                         (ltype, rtype) -- false when either is null
 *   SDH_OP_ARITH          pop r, l; push l (imm = SDH_AR_*) r in restype (the widest of D > F > L > I);
 *                         division and modulo by zero give null
 */
#ifndef SIDDHI_HIP_IR_H
#define SIDDHI_HIP_IR_H

#define SDH_IR_MAGIC "SDHIR001"
#define SDH_IR_VERSION 2

/* attribute / value types */
#define SDH_T_INT 0
#define SDH_T_LONG 1
#define SDH_T_FLOAT 2
#define SDH_T_DOUBLE 3
#define SDH_T_BOOL 4
#define SDH_T_STRING 5

/* bytecode */
#define SDH_OP_CONST 1
#define SDH_OP_ATTR 2
#define SDH_OP_IS_NULL 3
#define SDH_OP_STREAM_IS_NULL 4
#define SDH_OP_CMP 5
#define SDH_OP_AND 6
#define SDH_OP_OR 7
#define SDH_OP_NOT 8
#define SDH_OP_ARITH 9
#define SDH_CMP_EQ 0
#define SDH_CMP_NE 1
#define SDH_CMP_GT 2
#define SDH_CMP_GE 3
#define SDH_CMP_LT 4
#define SDH_CMP_LE 5
#define SDH_AR_ADD 0
#define SDH_AR_SUB 1
#define SDH_AR_MUL 2
#define SDH_AR_DIV 3
#define SDH_AR_MOD 4
#define SDH_IDX_CURRENT (-1)
#define SDH_IDX_LAST (-2)
#define SDH_INSN_W0(op, ltype, rtype, restype) \
  ((long long)(op) | ((long long)(ltype) << 8) | ((long long)(rtype) << 16) | ((long long)(restype) << 24))

/* states, queries, receivers, runtime nodes */
#define SDH_K_STREAM 0
#define SDH_K_COUNT 1
#define SDH_K_LOGICAL 2
#define SDH_K_ABSENT 3
#define SDH_L_AND 0
#define SDH_L_OR 1
#define SDH_Q_PATTERN 0
#define SDH_Q_SEQUENCE 1
#define SDH_R_SINGLE 0
#define SDH_R_MULTI 1
#define SDH_N_STREAM 0
#define SDH_N_NEXT 1
#define SDH_N_EVERY 2
#define SDH_N_LOGICAL 3
#define SDH_N_COUNT 4

#endif
