package wire

import (
	"bytes"
	"errors"
	"os"
	"path/filepath"
	"reflect"
	"testing"
)

// figure1.drw1 is written by tests/golden/make_wire_fixture.py through
// dag_rider_amd/wire.py: the Go encoder must reproduce it byte for byte.
func fixture(t *testing.T) []byte {
	t.Helper()
	b, err := os.ReadFile(filepath.Join("..", "..", "..", "tests", "golden", "figure1.drw1"))
	if err != nil {
		t.Fatal(err)
	}
	return b
}

func TestFigure1Fixture(t *testing.T) {
	buf := fixture(t)
	dag, err := Decode(buf)
	if err != nil {
		t.Fatal(err)
	}
	if len(dag) != 5 {
		t.Fatalf("rounds = %d, want 5", len(dag))
	}
	for r, rnd := range dag {
		if len(rnd) != 5 || rnd[0].ID != (ID{0, 0}) { // slot 0 of every round is the ghost {0,0}
			t.Fatalf("round %d: %d slots, slot 0 = %v", r, len(rnd), rnd[0].ID)
		}
	}
	v := dag[2][1]
	if v.ID != (ID{2, 1}) || string(v.Block) != "tx-batch" ||
		!reflect.DeepEqual(v.StrongEdges, []ID{{1, 1}, {1, 2}, {1, 4}}) {
		t.Fatalf("dag[2][1] = %+v", v)
	}
	w := dag[4][1] // Figure 1's weak edge (4,1) -> (2,4)
	if !reflect.DeepEqual(w.WeakEdges, []ID{{2, 4}}) || len(w.StrongEdges) != 3 {
		t.Fatalf("dag[4][1] = %+v", w)
	}
	if got := Encode(dag); !bytes.Equal(got, buf) {
		t.Fatalf("re-encoded capture differs from wire.py's (%d vs %d bytes)", len(got), len(buf))
	}
}

func TestCorruptRejected(t *testing.T) {
	buf := fixture(t)
	for cut := 0; cut < len(buf); cut += 7 {
		if _, err := Decode(buf[:cut]); !errors.Is(err, ErrCorrupt) {
			t.Fatalf("truncated at %d: err = %v", cut, err)
		}
	}
	if _, err := Decode(append(append([]byte(nil), buf...), 0)); !errors.Is(err, ErrCorrupt) {
		t.Fatal("trailing byte accepted")
	}
	bad := append([]byte(nil), buf...)
	copy(bad, "XXXX")
	if _, err := Decode(bad); !errors.Is(err, ErrCorrupt) {
		t.Fatal("bad magic accepted")
	}
}

func TestFlattenDoesNotAliasEdges(t *testing.T) {
	strong := make([]ID, 2, 8) // spare capacity: an append(strong, weak...) would write into it
	strong[0], strong[1] = ID{1, 1}, ID{1, 2}
	vs := []Vertex{{ID: ID{2, 3}, StrongEdges: strong, WeakEdges: []ID{{0, 4}}}}
	ids, off, preds := Preds(vs)
	if !reflect.DeepEqual(ids, []int32{2, 3}) || !reflect.DeepEqual(off, []uint32{0, 3}) ||
		!reflect.DeepEqual(preds, []int32{1, 1, 1, 2, 0, 4}) {
		t.Fatalf("Preds = %v %v %v", ids, off, preds)
	}
	if full := strong[:cap(strong)]; full[2] != (ID{}) {
		t.Fatal("Preds wrote into the caller's strong-edge backing array")
	}
	b, err := FlattenBatch(vs, nil)
	if err != nil || !reflect.DeepEqual(b.SlotRound, []int32{2}) || !reflect.DeepEqual(b.WeakIDs, []int32{0, 4}) {
		t.Fatalf("FlattenBatch = %+v, %v", b, err)
	}
	if _, err := FlattenBatch(vs, []int{1, 2}); err == nil {
		t.Fatal("mismatched slotRound accepted")
	}
}
