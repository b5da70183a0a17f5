package dagridergpu

import (
	"os"
	"path/filepath"
	"testing"

	"github.com/xenowits/dag-rider/dagridergpu/wire"
)

// The reference's TestPath cases (process_internal_test.go:20-83) on the
// Figure-1 DAG, loaded from the DRW1 fixture through the library's C reader,
// then vertex by vertex through AppendVertices.  Needs a gfx950 device and the
// built library (make lib); skipped without a device.
func figure1(t *testing.T) (*Mirror, [][]wire.Vertex, []byte) {
	t.Helper()
	buf, err := os.ReadFile(filepath.Join("..", "..", "tests", "golden", "figure1.drw1"))
	if err != nil {
		t.Fatal(err)
	}
	dag, err := wire.Decode(buf)
	if err != nil {
		t.Fatal(err)
	}
	m, err := New(4, 1, 16, 0)
	if err != nil {
		t.Skipf("no device: %v", err)
	}
	return m, dag, buf
}

var testPath = []struct {
	from, to wire.ID
	strong   bool
	want     bool
}{
	{wire.ID{3, 1}, wire.ID{2, 3}, true, true},   // process_internal_test.go:20-31
	{wire.ID{3, 3}, wire.ID{1, 4}, true, true},   // :33-44
	{wire.ID{4, 1}, wire.ID{2, 4}, false, true},  // :46-57
	{wire.ID{4, 1}, wire.ID{1, 1}, false, true},  // :59-70
	{wire.ID{3, 3}, wire.ID{2, 4}, false, false}, // :72-83
}

func TestPathFromCapture(t *testing.T) {
	m, _, buf := figure1(t)
	defer m.Close()
	if err := m.AppendCapture(buf); err != nil {
		t.Fatal(err)
	}
	for _, c := range testPath {
		if got := m.Path(c.from, c.to, c.strong); got != c.want {
			t.Errorf("path(%v, %v, %v) = %v, want %v", c.from, c.to, c.strong, got, c.want)
		}
	}
}

func TestPathVertexByVertex(t *testing.T) {
	m, dag, _ := figure1(t)
	defer m.Close()
	for r, rnd := range dag {
		for _, v := range rnd {
			if err := m.AppendVertices([]wire.Vertex{v}, []int{r}); err != nil {
				t.Fatal(err)
			}
		}
	}
	for _, c := range testPath {
		if got := m.Path(c.from, c.to, c.strong); got != c.want {
			t.Errorf("path(%v, %v, %v) = %v, want %v", c.from, c.to, c.strong, got, c.want)
		}
	}
	// waveReady(1) on Figure 1: leader (1,1), one strong voter in round 4, no commit
	commit, vcount, _, err := m.WaveReady(1, 0)
	if err != nil || commit || vcount != 1 {
		t.Fatalf("WaveReady(1) = %v %d %v", commit, vcount, err)
	}
}
