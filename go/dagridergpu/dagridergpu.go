// Package dagridergpu binds the MI355X causal-history engine
// (include/dagrider_gpu.h, dag_rider_amd/libdagrider_gpu.so) for the
// reference's process package: one Mirror per Process holds a device copy of
// p.dag (process/process.go:79) and answers path (:89-148), waveReady
// (:314-354), getWaveVertexLeader/chooseLeader (:357-392), orderVertices
// (:404-443) and the buffer loop's present() (:200-234, :374-384).
//
// Memory (cgo pointer rules): the append and query calls pass Go slices of
// C-compatible scalars (int32, uint32, uint8) straight to C.  That is allowed
// because that memory holds no Go pointers, and the library keeps no host
// pointer after a call returns.  Replay's output struct carries pointers, so its
// arrays are C.malloc'd and copied out.
//
// Errors: DR_E_INVAL is where process.go would panic (an index out of range, an
// empty Pop); the methods that stand in for a panicking Go function panic
// with the library's message, the others return it as an error.
//
// Threading: calls on one Mirror must be serialised, as the reference's single
// Start goroutine serialises its p.dag mutations.  Each call selects its own
// HIP device, so runtime.LockOSThread is not needed.
package dagridergpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../dag_rider_amd -ldagrider_gpu -Wl,-rpath,${SRCDIR}/../../dag_rider_amd
#include <stdlib.h>
#include "dagrider_gpu.h"
#include "dagrider_wire.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"

	"github.com/xenowits/dag-rider/dagridergpu/wire"
)

// Chain, delivery and weak-edge modes (include/dagrider_gpu.h).
const (
	ChainLiteral    = int(C.DR_CHAIN_LITERAL)    // decidedWave stays 0 (the code as written)
	ChainPersistent = int(C.DR_CHAIN_PERSISTENT) // decidedWave advances (Alg. 3)
	DeliverRef      = int(C.DR_DELIVER_REF)      // every reachable vertex per pop (process.go:423-427)
	DeliverPaper    = int(C.DR_DELIVER_PAPER)    // each vertex once per call (Alg. 3 line 54)
	WeakLiteral     = int(C.DR_WEAK_LITERAL)
	WeakPaper       = int(C.DR_WEAK_PAPER)
	LeaderConst1    = int(C.DR_LEADER_CONST1) // chooseLeader as written: process 1
	LeaderSeeded    = int(C.DR_LEADER_SEEDED)
	LeaderTable     = int(C.DR_LEADER_TABLE)
)

// Mirror is one device copy of a Process's DAG (one dr_ctx).
type Mirror struct {
	ctx *C.dr_ctx
	ids []int32 // OrderVertices' id buffer, reused and grown across calls
}

// Error is a non-panicking library failure.
type Error struct {
	Code int
	Msg  string
}

func (e *Error) Error() string { return fmt.Sprintf("dagridergpu: %s (status %d)", e.Msg, e.Code) }

// ErrCapacity is wrapped by errors for an output the caller sized too small.
var ErrCapacity = errors.New("output capacity")

// New is New(index, faulty, tp) (process.go:34-60) for the mirror: n processes,
// f faulty, room for maxRounds rounds, on HIP device `device`.
func New(n, faulty, maxRounds, device int) (*Mirror, error) {
	var c *C.dr_ctx
	if rc := C.dr_create(C.int(n), C.int(faulty), C.int(maxRounds), C.int(device), &c); rc != C.DR_OK {
		return nil, &Error{int(rc), C.GoString(C.dr_last_error(nil))}
	}
	return &Mirror{ctx: c}, nil
}

// Close releases the device mirror.
func (m *Mirror) Close() {
	if m.ctx != nil {
		C.dr_destroy(m.ctx)
		m.ctx = nil
	}
}

func (m *Mirror) fail(rc C.int) error {
	if rc == C.DR_OK {
		return nil
	}
	e := &Error{int(rc), C.GoString(C.dr_last_error(m.ctx))}
	if rc == C.DR_E_CAPACITY {
		return fmt.Errorf("%w: %v", ErrCapacity, e)
	}
	return e
}

// must is fail for the calls whose Go original panics: DR_E_INVAL panics.
func (m *Mirror) must(rc C.int) error {
	if rc == C.DR_E_INVAL {
		panic("runtime error: " + C.GoString(C.dr_last_error(m.ctx)))
	}
	return m.fail(rc)
}

// C views of Go scalar slices; an empty slice passes one zero element (the
// library never reads it) so that no call sees a null array.
func i32p(a []int32) *C.int32_t {
	if len(a) == 0 {
		a = []int32{0, 0}
	}
	return (*C.int32_t)(unsafe.Pointer(&a[0]))
}

func u32p(a []uint32) *C.uint32_t {
	if len(a) == 0 {
		a = []uint32{0}
	}
	return (*C.uint32_t)(unsafe.Pointer(&a[0]))
}

func idPairs(ids []wire.ID) []int32 {
	o := make([]int32, 0, 2*len(ids))
	for _, v := range ids {
		o = append(o, int32(v.Round), int32(v.Source))
	}
	return o
}

// NumRounds is len(p.dag) as mirrored.
func (m *Mirror) NumRounds() int { return int(C.dr_num_rounds(m.ctx)) }

// AppendRounds mirrors whole new rounds: p.dag = append(p.dag, rounds...).
func (m *Mirror) AppendRounds(rounds [][]wire.Vertex) error {
	f := wire.FlattenRounds(rounds)
	return m.fail(C.dr_append_rounds_lists(m.ctx, C.int(m.NumRounds()), C.int(len(rounds)), u32p(f.SlotOff),
		i32p(f.SlotID), u32p(f.StrongOff), i32p(f.StrongIDs), u32p(f.WeakOff), i32p(f.WeakIDs)))
}

// AppendVertices is p.dag[v.id.round] = append(p.dag[v.id.round], v)
// (process.go:229) for each vertex in order, into any mirrored round; a round
// index == NumRounds() opens it.  slotRound may be nil (the vertex's own round).
// All or nothing.  An index past the end panics, as the Go index does.
func (m *Mirror) AppendVertices(vs []wire.Vertex, slotRound []int) error {
	if len(vs) == 0 {
		return nil
	}
	b, err := wire.FlattenBatch(vs, slotRound)
	if err != nil {
		return err
	}
	return m.must(C.dr_append_vertices(m.ctx, C.int(len(vs)), i32p(b.SlotRound), i32p(b.IDs), u32p(b.StrongOff),
		i32p(b.StrongIDs), u32p(b.WeakOff), i32p(b.WeakIDs)))
}

// AppendCapture appends every round of a DRW1 capture (wire.Encode) through the
// library's C reader, which checks every size and offset first.
func (m *Mirror) AppendCapture(buf []byte) error {
	if len(buf) == 0 {
		return m.fail(C.DR_E_INVAL)
	}
	return m.fail(C.dr_wire_append(m.ctx, unsafe.Pointer(&buf[0]), C.size_t(len(buf))))
}

// Path is path(from, to, strongPath) (process.go:89-148).
func (m *Mirror) Path(from, to wire.ID, strongPath bool) bool {
	out, err := m.PathBatch([]wire.ID{from}, []wire.ID{to}, strongPath)
	if err != nil {
		panic(err)
	}
	return out[0]
}

// PathBatch answers many path queries in one device call.
func (m *Mirror) PathBatch(from, to []wire.ID, strongPath bool) ([]bool, error) {
	if len(from) != len(to) {
		return nil, fmt.Errorf("dagridergpu: %d sources for %d targets", len(from), len(to))
	}
	if len(from) == 0 {
		return nil, nil
	}
	s := C.int(0)
	if strongPath {
		s = 1
	}
	res := make([]uint8, len(from))
	if err := m.must(C.dr_path_batch(m.ctx, C.int(len(from)), i32p(idPairs(from)), i32p(idPairs(to)), s,
		(*C.uint8_t)(unsafe.Pointer(&res[0])))); err != nil {
		return nil, err
	}
	out := make([]bool, len(res))
	for i, x := range res {
		out[i] = x != 0
	}
	return out, nil
}

// SetLeaderCoin selects chooseLeader (process.go:386-392): LeaderConst1 (the
// reference), LeaderSeeded (dr_coin_leader(seed, w, n)) or LeaderTable
// (table[w-1], 1 beyond it).
func (m *Mirror) SetLeaderCoin(mode int, seed uint64, table []int) error {
	t := make([]int32, len(table))
	for i, x := range table {
		t[i] = int32(x)
	}
	return m.fail(C.dr_set_leader_coin(m.ctx, C.int(mode), C.uint64_t(seed), C.int(len(t)), i32p(t)))
}

// WaveLeader is chooseLeader(wave) as the mirror decides it; the leader vertex
// of getWaveVertexLeader (process.go:357-371) is (round(wave,1), WaveLeader).
func (m *Mirror) WaveLeader(wave int) int { return int(C.dr_wave_leader(m.ctx, C.int(wave))) }

// ReplayGraphState is the form of the mirror's last Replay (dr_replay_graph_state): 1 = the
// captured hipGraph was launched (DR_OPT_REPLAY_GRAPH), 0 = kernel by kernel, -1 = kernel by
// kernel after a failed capture.
func (m *Mirror) ReplayGraphState() int { return int(C.dr_replay_graph_state(m.ctx)) }

// WaveReady is waveReady(wave) (process.go:314-354) given decidedWave: the
// commit decision, the vote count (-1: no leader vertex) and on commit the
// waves whose leaders are pushed onto leadersStack, in push order.
func (m *Mirror) WaveReady(wave, decidedWave int) (commit bool, vcount int, pushed []int, err error) {
	var c C.uint8_t
	var vc C.int32_t
	var np C.int
	buf := make([]int32, wave+1)
	if err = m.must(C.dr_wave_ready(m.ctx, C.int(wave), C.int(decidedWave), &c, &vc, i32p(buf), C.int(len(buf)),
		&np)); err != nil {
		return
	}
	for i := 0; i < int(np); i++ {
		pushed = append(pushed, int(buf[i]))
	}
	return c != 0, int(vc), pushed, nil
}

// OrderVertices is orderVertices() (process.go:404-443) with leadersStack =
// stack (bottom to top) and p.round = pRound: the delivered ids in order (the
// caller forwards each to p.tp.Broadcast as :433-441 does).
func (m *Mirror) OrderVertices(stack []wire.ID, pRound, mode int) ([]wire.ID, error) {
	st := idPairs(stack)
	if len(m.ids) == 0 {
		m.ids = make([]int32, 2*4096)
	}
	var n C.size_t
	// one call into the reused buffer; only an undersized buffer (DR_E_CAPACITY,
	// n = the total) costs a second, exactly sized call
	rc := C.dr_order_vertices(m.ctx, i32p(st), C.int(len(stack)), C.int(pRound), C.int(mode), i32p(m.ids),
		C.size_t(len(m.ids)/2), &n, nil, nil)
	if rc == C.DR_E_CAPACITY {
		m.ids = make([]int32, 2*int(n))
		rc = C.dr_order_vertices(m.ctx, i32p(st), C.int(len(stack)), C.int(pRound), C.int(mode), i32p(m.ids),
			n, &n, nil, nil)
	}
	if err := m.must(rc); err != nil {
		return nil, err
	}
	out := make([]wire.ID, n)
	for i := range out {
		out[i] = wire.ID{Round: int(m.ids[2*i]), Source: int(m.ids[2*i+1])}
	}
	return out, nil
}

// SetWeakEdges is setWeakEdges(v, round) (process.go:298-310) for a vertex of
// `round` with the given strong edges: the ids that become its weak edges.
func (m *Mirror) SetWeakEdges(round int, strong []wire.ID, mode int) ([]wire.ID, error) {
	s := idPairs(strong)
	var n C.size_t
	rc := C.dr_set_weak_edges(m.ctx, C.int(round), C.int(len(strong)), i32p(s), C.int(mode), nil, 0, &n)
	if rc != C.DR_OK && rc != C.DR_E_CAPACITY {
		return nil, m.must(rc)
	}
	if n == 0 {
		return nil, nil
	}
	ids := make([]int32, 2*int(n))
	if err := m.must(C.dr_set_weak_edges(m.ctx, C.int(round), C.int(len(strong)), i32p(s), C.int(mode), i32p(ids), n,
		&n)); err != nil {
		return nil, err
	}
	out := make([]wire.ID, n)
	for i := range out {
		out[i] = wire.ID{Round: int(ids[2*i]), Source: int(ids[2*i+1])}
	}
	return out, nil
}

// AdmitBuffer is one pass of the buffer loop (process.go:200-234): admit[i]
// when every predecessor of buffer[i] is present() (process.go:374-384) or was
// admitted earlier in the pass.  The caller appends the admitted vertices
// (AppendVertices, buffer order) and keeps the rest.  Panics where the pass
// would (present() past the end of p.dag).
func (m *Mirror) AdmitBuffer(pRound int, buffer []wire.Vertex) ([]bool, error) {
	if len(buffer) == 0 {
		return nil, nil
	}
	ids, off, preds := wire.Preds(buffer) // strong and weak edges copied, never appended in place
	adm := make([]uint8, len(buffer))
	if err := m.must(C.dr_buffer_admit(m.ctx, C.int(pRound), C.int(len(buffer)), i32p(ids), u32p(off), i32p(preds),
		(*C.uint8_t)(unsafe.Pointer(&adm[0])))); err != nil {
		return nil, err
	}
	out := make([]bool, len(adm))
	for i, x := range adm {
		out[i] = x != 0
	}
	return out, nil
}

// ReplayResult is dr_replay_out without the pointers.
type ReplayResult struct {
	Commit                               []bool
	VCount                               []int
	PushOff                              []uint32
	PushWave                             []int
	PopCount, PopDigest, PopEdges        []uint64
	CommitEdges, ChainEdges, DeliverEdges uint64
}

// Replay runs waveReady(w) for w = 1..nwaves and orderVertices on each commit
// (the wiring process.go:325 leaves out), entirely on the device.
func (m *Mirror) Replay(nwaves, chainMode, deliverMode int) (*ReplayResult, error) {
	pushCap := 2*nwaves + 1
	if chainMode == ChainLiteral {
		pushCap = nwaves * (nwaves + 1) / 2
	}
	if pushCap < 1 {
		pushCap = 1
	}
	// the struct holds pointers: its arrays live in C memory (cgo rules)
	alloc := func(n int) unsafe.Pointer { return C.calloc(C.size_t(n), 1) }
	cm, vc := alloc(nwaves), alloc(4*nwaves)
	po, pw := alloc(4*(nwaves+1)), alloc(4*pushCap)
	pc, pd, pe := alloc(8*pushCap), alloc(8*pushCap), alloc(8*pushCap)
	defer func() {
		for _, p := range []unsafe.Pointer{cm, vc, po, pw, pc, pd, pe} {
			C.free(p)
		}
	}()
	if cm == nil || vc == nil || po == nil || pw == nil || pc == nil || pd == nil || pe == nil {
		return nil, errors.New("dagridergpu: out of host memory")
	}
	var o C.dr_replay_out
	o.commit, o.vcount = (*C.uint8_t)(cm), (*C.int32_t)(vc)
	o.push_off, o.push_wave, o.push_cap = (*C.uint32_t)(po), (*C.int32_t)(pw), C.int64_t(pushCap)
	o.pop_count, o.pop_digest, o.pop_edges = (*C.uint64_t)(pc), (*C.uint64_t)(pd), (*C.uint64_t)(pe)
	if err := m.fail(C.dr_replay(m.ctx, C.int(nwaves), C.int(chainMode), C.int(deliverMode), &o)); err != nil {
		return nil, err
	}
	np := int(o.n_push)
	r := &ReplayResult{CommitEdges: uint64(o.commit_edges), ChainEdges: uint64(o.chain_edges),
		DeliverEdges: uint64(o.deliver_edges)}
	cms := unsafe.Slice((*uint8)(cm), nwaves)
	vcs := unsafe.Slice((*int32)(vc), nwaves)
	for w := 0; w < nwaves; w++ {
		r.Commit = append(r.Commit, cms[w] != 0)
		r.VCount = append(r.VCount, int(vcs[w]))
	}
	r.PushOff = append(r.PushOff, unsafe.Slice((*uint32)(po), nwaves+1)...)
	for _, x := range unsafe.Slice((*int32)(pw), np) {
		r.PushWave = append(r.PushWave, int(x))
	}
	r.PopCount = append(r.PopCount, unsafe.Slice((*uint64)(pc), np)...)
	r.PopDigest = append(r.PopDigest, unsafe.Slice((*uint64)(pd), np)...)
	r.PopEdges = append(r.PopEdges, unsafe.Slice((*uint64)(pe), np)...)
	return r, nil
}
