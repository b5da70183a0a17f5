// Package wire holds the pure-Go half of the dag-rider GPU binding: the flat
// array forms of a [][]vertex that the C ABI's append calls take
// (include/dagrider_gpu.h dr_append_rounds_lists, dr_append_vertices) and the
// DRW1 capture format (include/dagrider_wire.h, dag_rider_amd/wire.py).
//
// It has no cgo and no device dependency, so it builds and tests anywhere.  The
// reference moves vertices between processes as Go values over channels
// (bcastMsg, process/transport.go:13-17, carrying vertex, process/process.go:26-31)
// and has no on-disk form; DRW1 stores exactly the arrays the mirror appends.
package wire

import (
	"encoding/binary"
	"errors"
	"fmt"
)

// ID is vertexID (process/process.go:20-23).
type ID struct {
	Round  int
	Source int
}

// Vertex is vertex (process/process.go:26-31) with exported fields.
type Vertex struct {
	ID          ID
	Block       []byte
	StrongEdges []ID
	WeakEdges   []ID
}

// Rounds is the array form of dr_append_rounds_lists: whole rounds, slots in
// insertion order.  Id arrays hold (round, source) pairs.
type Rounds struct {
	SlotOff   []uint32 // nrounds+1
	SlotID    []int32  // 2 per slot
	StrongOff []uint32 // nslots+1
	StrongIDs []int32  // 2 per strong edge
	WeakOff   []uint32 // nslots+1
	WeakIDs   []int32  // 2 per weak edge
}

// NumSlots is the number of vertices (slots) in r.
func (r *Rounds) NumSlots() int { return len(r.SlotID) / 2 }

// FlattenRounds flattens rounds (p.dag[r0:r1] of the reference) into the
// dr_append_rounds_lists arrays.  Each vertex's strong and weak edges are
// copied out one by one: the caller's edge slices are never appended to.
func FlattenRounds(rounds [][]Vertex) Rounds {
	f := Rounds{SlotOff: []uint32{0}, StrongOff: []uint32{0}, WeakOff: []uint32{0}}
	for _, rnd := range rounds {
		for i := range rnd {
			v := &rnd[i]
			f.SlotID = append(f.SlotID, int32(v.ID.Round), int32(v.ID.Source))
			for _, e := range v.StrongEdges {
				f.StrongIDs = append(f.StrongIDs, int32(e.Round), int32(e.Source))
			}
			for _, e := range v.WeakEdges {
				f.WeakIDs = append(f.WeakIDs, int32(e.Round), int32(e.Source))
			}
			f.StrongOff = append(f.StrongOff, uint32(len(f.StrongIDs)/2))
			f.WeakOff = append(f.WeakOff, uint32(len(f.WeakIDs)/2))
		}
		f.SlotOff = append(f.SlotOff, uint32(len(f.SlotID)/2))
	}
	return f
}

// Batch is the array form of dr_append_vertices: k vertices, each appended to
// p.dag[SlotRound[i]] in order (process.go:229).
type Batch struct {
	SlotRound []int32 // the round index per vertex (the Go index of p.dag)
	IDs       []int32 // 2 per vertex
	StrongOff []uint32
	StrongIDs []int32
	WeakOff   []uint32
	WeakIDs   []int32
}

// FlattenBatch flattens vertices for dr_append_vertices.  slotRound may be nil:
// each vertex then goes to p.dag[v.ID.Round], as process.go:229 indexes it.
func FlattenBatch(vs []Vertex, slotRound []int) (Batch, error) {
	if slotRound != nil && len(slotRound) != len(vs) {
		return Batch{}, fmt.Errorf("wire: %d rounds for %d vertices", len(slotRound), len(vs))
	}
	b := Batch{StrongOff: []uint32{0}, WeakOff: []uint32{0}}
	for i := range vs {
		v := &vs[i]
		r := v.ID.Round
		if slotRound != nil {
			r = slotRound[i]
		}
		b.SlotRound = append(b.SlotRound, int32(r))
		b.IDs = append(b.IDs, int32(v.ID.Round), int32(v.ID.Source))
		for _, e := range v.StrongEdges {
			b.StrongIDs = append(b.StrongIDs, int32(e.Round), int32(e.Source))
		}
		for _, e := range v.WeakEdges {
			b.WeakIDs = append(b.WeakIDs, int32(e.Round), int32(e.Source))
		}
		b.StrongOff = append(b.StrongOff, uint32(len(b.StrongIDs)/2))
		b.WeakOff = append(b.WeakOff, uint32(len(b.WeakIDs)/2))
	}
	return b, nil
}

// Preds flattens the buffer for dr_buffer_admit: ids and every predecessor
// (strong then weak edges) per vertex, without touching the vertices' slices.
func Preds(buffer []Vertex) (ids []int32, off []uint32, preds []int32) {
	off = []uint32{0}
	for i := range buffer {
		v := &buffer[i]
		ids = append(ids, int32(v.ID.Round), int32(v.ID.Source))
		for _, e := range v.StrongEdges {
			preds = append(preds, int32(e.Round), int32(e.Source))
		}
		for _, e := range v.WeakEdges {
			preds = append(preds, int32(e.Round), int32(e.Source))
		}
		off = append(off, uint32(len(preds)/2))
	}
	return ids, off, preds
}

// Magic starts every DRW1 capture.
const Magic = "DRW1"

// ErrCorrupt is returned (wrapped) for a truncated or inconsistent capture.
var ErrCorrupt = errors.New("corrupt DRW1 capture")

// Encode writes rounds as a DRW1 capture (little-endian): magic, u32 nrounds,
// u32 nslots; the six Rounds arrays, each preceded by its u64 element count;
// block_off u64[nslots+1]; the block bytes.  Byte-identical to
// dag_rider_amd/wire.py encode().
func Encode(rounds [][]Vertex) []byte {
	f := FlattenRounds(rounds)
	ns := f.NumSlots()
	out := make([]byte, 0, 64+4*(len(f.SlotOff)+len(f.SlotID)+len(f.StrongOff)+len(f.StrongIDs)+
		len(f.WeakOff)+len(f.WeakIDs))+8*(ns+1))
	out = append(out, Magic...)
	out = binary.LittleEndian.AppendUint32(out, uint32(len(rounds)))
	out = binary.LittleEndian.AppendUint32(out, uint32(ns))
	u32s := func(a []uint32) {
		out = binary.LittleEndian.AppendUint64(out, uint64(len(a)))
		for _, x := range a {
			out = binary.LittleEndian.AppendUint32(out, x)
		}
	}
	i32s := func(a []int32) {
		out = binary.LittleEndian.AppendUint64(out, uint64(len(a)))
		for _, x := range a {
			out = binary.LittleEndian.AppendUint32(out, uint32(x))
		}
	}
	u32s(f.SlotOff)
	i32s(f.SlotID)
	u32s(f.StrongOff)
	i32s(f.StrongIDs)
	u32s(f.WeakOff)
	i32s(f.WeakIDs)
	var boff uint64
	out = binary.LittleEndian.AppendUint64(out, 0)
	for _, rnd := range rounds {
		for i := range rnd {
			boff += uint64(len(rnd[i].Block))
			out = binary.LittleEndian.AppendUint64(out, boff)
		}
	}
	for _, rnd := range rounds {
		for i := range rnd {
			out = append(out, rnd[i].Block...)
		}
	}
	return out
}

type reader struct {
	b   []byte
	pos int
}

func (r *reader) take(n uint64) ([]byte, error) {
	if n > uint64(len(r.b)-r.pos) {
		return nil, fmt.Errorf("%w: truncated", ErrCorrupt)
	}
	s := r.b[r.pos : r.pos+int(n)]
	r.pos += int(n)
	return s, nil
}

func (r *reader) words() ([]uint32, error) {
	h, err := r.take(8)
	if err != nil {
		return nil, err
	}
	k := binary.LittleEndian.Uint64(h)
	if k > uint64(len(r.b)-r.pos)/4 {
		return nil, fmt.Errorf("%w: array runs past the end", ErrCorrupt)
	}
	s, _ := r.take(4 * k)
	a := make([]uint32, k)
	for i := range a {
		a[i] = binary.LittleEndian.Uint32(s[4*i:])
	}
	return a, nil
}

func asInt32(a []uint32) []int32 {
	o := make([]int32, len(a))
	for i, x := range a {
		o[i] = int32(x)
	}
	return o
}

// prefix checks an offset array: n+1 entries, 0-based, non-decreasing, ending at total.
func prefix(name string, off []uint32, n, total int) error {
	if len(off) != n+1 || off[0] != 0 || int(off[n]) != total {
		return fmt.Errorf("%w: %s is not a 0-based prefix of %d entries ending at %d", ErrCorrupt, name, n+1, total)
	}
	for i := 1; i <= n; i++ {
		if off[i] < off[i-1] {
			return fmt.Errorf("%w: %s decreases at %d", ErrCorrupt, name, i)
		}
	}
	return nil
}

// Parse checks every size and offset of a capture (as dr_wire_check does) and
// returns its arrays plus the block offsets and bytes.
func Parse(buf []byte) (f Rounds, nrounds int, boff []uint64, blocks []byte, err error) {
	r := &reader{b: buf}
	h, err := r.take(12)
	if err != nil || string(h[:4]) != Magic {
		return f, 0, nil, nil, fmt.Errorf("%w: not a DRW1 capture", ErrCorrupt)
	}
	nrounds = int(binary.LittleEndian.Uint32(h[4:]))
	ns := int(binary.LittleEndian.Uint32(h[8:]))
	var arr [6][]uint32
	for i := range arr {
		if arr[i], err = r.words(); err != nil {
			return f, 0, nil, nil, err
		}
	}
	f = Rounds{SlotOff: arr[0], SlotID: asInt32(arr[1]), StrongOff: arr[2], StrongIDs: asInt32(arr[3]),
		WeakOff: arr[4], WeakIDs: asInt32(arr[5])}
	if len(f.SlotID) != 2*ns || len(f.StrongIDs)%2 != 0 || len(f.WeakIDs)%2 != 0 {
		return f, 0, nil, nil, fmt.Errorf("%w: array sizes disagree with the header", ErrCorrupt)
	}
	if err = prefix("slot_off", f.SlotOff, nrounds, ns); err != nil {
		return
	}
	if err = prefix("strong_off", f.StrongOff, ns, len(f.StrongIDs)/2); err != nil {
		return
	}
	if err = prefix("weak_off", f.WeakOff, ns, len(f.WeakIDs)/2); err != nil {
		return
	}
	bs, err := r.take(8 * uint64(ns+1))
	if err != nil {
		return
	}
	boff = make([]uint64, ns+1)
	for i := range boff {
		boff[i] = binary.LittleEndian.Uint64(bs[8*i:])
		if (i == 0 && boff[0] != 0) || (i > 0 && boff[i] < boff[i-1]) {
			return f, 0, nil, nil, fmt.Errorf("%w: block offsets", ErrCorrupt)
		}
	}
	if boff[ns] != uint64(len(buf)-r.pos) {
		return f, 0, nil, nil, fmt.Errorf("%w: block bytes truncated or trailing data", ErrCorrupt)
	}
	return f, nrounds, boff, buf[r.pos:], nil
}

// Decode reads a capture back into rounds (blocks are copied out of buf).
func Decode(buf []byte) ([][]Vertex, error) {
	f, nrounds, boff, blocks, err := Parse(buf)
	if err != nil {
		return nil, err
	}
	ids := func(a []int32, lo, hi uint32) []ID {
		var o []ID
		for e := lo; e < hi; e++ {
			o = append(o, ID{int(a[2*e]), int(a[2*e+1])})
		}
		return o
	}
	out := make([][]Vertex, nrounds)
	k := 0
	for r := 0; r < nrounds; r++ {
		for ; k < int(f.SlotOff[r+1]); k++ {
			v := Vertex{
				ID:          ID{int(f.SlotID[2*k]), int(f.SlotID[2*k+1])},
				Block:       append([]byte(nil), blocks[boff[k]:boff[k+1]]...),
				StrongEdges: ids(f.StrongIDs, f.StrongOff[k], f.StrongOff[k+1]),
				WeakEdges:   ids(f.WeakIDs, f.WeakOff[k], f.WeakOff[k+1]),
			}
			out[r] = append(out[r], v)
		}
	}
	return out, nil
}
