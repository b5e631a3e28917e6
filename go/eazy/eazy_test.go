package eazy

// A few of the reference's known answers (eazy_test.go), for a Go box with an
// MI355X: go test ./go/eazy

import (
	"bytes"
	"io"
	"runtime"
	"testing"
)

func TestMagic(t *testing.T) { // eazy_test.go:39-64
	var buf bytes.Buffer
	w := NewWriter(&buf, MiB, 512)
	if err := w.WriteHeader(); err != nil {
		t.Fatal(err)
	}
	if !bytes.Equal(buf.Bytes(), []byte{0x80, 0x02, 'e', 'a', 'z', 'y', 0x80, 0x10, 0x14}) {
		t.Fatalf("header % x", buf.Bytes())
	}
}

func TestCopy(t *testing.T) { // eazy_test.go:106-183
	var buf bytes.Buffer
	w := NewWriter(&buf, 32, 16)
	w.AppendMagic = false
	w.Write([]byte("prefix_1234_suffix"))
	st := buf.Len()
	w.Write([]byte("prefix_567_suffix"))
	want := append([]byte{Copy | 7, 0x12 - 7, Literal | 3}, "567"...)
	want = append(want, Copy|7, 0x11-7)
	if !bytes.Equal(buf.Bytes()[st:], want) {
		t.Fatalf("second write % x", buf.Bytes()[st:])
	}
	r := NewReaderBytes(buf.Bytes())
	p := make([]byte, 40)
	n, err := r.Read(p)
	if err != io.EOF || string(p[:n]) != "prefix_1234_suffixprefix_567_suffix" {
		t.Fatalf("read %q %v", p[:n], err)
	}
}

func TestCompressBatch(t *testing.T) {
	bufs := [][]byte{[]byte("level=info path=/api/v1 level=info path=/api/v2"), {}, bytes.Repeat([]byte("ab"), 3000)}
	for _, devs := range [][]int{nil, {0, 0}, {0, 0, 0}} { // every device; two and three shards on device 0
		Devices = devs
		got, err := CompressBatch(bufs, MiB, 1024)
		if err != nil {
			t.Fatal(err)
		}
		for k, p := range bufs {
			var buf bytes.Buffer
			NewWriter(&buf, MiB, 1024).Write(p)
			if len(p) > 0 && !bytes.Equal(got[k], buf.Bytes()) {
				t.Fatalf("devices %v: stream %d differs", devs, k)
			}
		}
	}
	Devices = nil
}

// The reference's error and panic values, text included (reader.go:57-76, 303, 319;
// writer.go:163, 167, 562, 596, 601).
func TestErrorText(t *testing.T) {
	for _, c := range []struct {
		err  error
		want string
	}{
		{ErrBlockSizeOverLimit, "block size is more than the limit"},
		{ErrUnsupportedMeta, "unsupported meta tag"},
		{ErrUnsupportedVersion, "unsupported file format version"},
		{ErrBreak, "break point"},
		{toErr(C_EUNSUPMETA, 0x28), "unsupported meta tag: 0x28"},
		{toErr(C_EUNSUPVER, 1), "unsupported file format version: 1"},
	} {
		if c.err.Error() != c.want {
			t.Errorf("%q, want %q", c.err.Error(), c.want)
		}
	}
	expectPanic := func(want interface{}, f func()) {
		defer func() {
			if r := recover(); r != want {
				t.Errorf("panic %v, want %v", r, want)
			}
		}()
		f()
	}
	expectPanic("block size must be a power of two (32 < bs < 1<<31)", func() { NewWriter(nil, 31, 16) })
	expectPanic("hash table size must be a power of two (hs >= 4)", func() { NewWriter(nil, 1024, 3) })
	expectPanic("too big length", func() { Encoder{}.Tag(nil, Literal, 0x1_1000_0000) })
	expectPanic("too big offset", func() { Encoder{}.Offset(nil, 0x1_1000_0000, 10) })
	expectPanic(1024, func() { Encoder{}.Meta(nil, 1024, 4) })
}

// Dump's text on the TestCopy stream (block 32, htable 16, no magic), whole and cut inside the
// second literal: the expected strings are eazy_amd/dump.py's (the C++ mirror prints the same,
// tests/test_cpp.py), which restates the reference's format (reader.go:602-732).
func TestDump(t *testing.T) {
	var buf bytes.Buffer
	w := NewWriter(&buf, 32, 16)
	w.AppendMagic = false
	w.Write([]byte("prefix_1234_suffix"))
	w.Write([]byte("prefix_567_suffix"))
	c := buf.Bytes()
	want := "     0     0       0  meta  2 1  \"\\x05\"    05\n" +
		"     3     3       0  lit    12        \"prefix_1234_suffix\"\n" +
		"    16    16      12  copy    7  off   12\n" +
		"    18    18      19  lit     3        \"567\"\n" +
		"    1c    1c      1c  copy    7  off   11\n" +
		"    1e     0      23  "
	if got := Dump(c); got != want {
		t.Fatalf("Dump:\n%q\nwant\n%q", got, want)
	}
	cut := "     0     0       0  meta  2 1  \"\\x05\"    05\n" +
		"     3     3       0  lit    12        \"prefix_1234_suffix\"\n" +
		"    16    16      12  copy    7  off   12\n" +
		"    18    18      19      19     0      19  \nerror: short buffer"
	if got := Dump(c[:len(c)-3]); got != cut {
		t.Fatalf("Dump (cut):\n%q\nwant\n%q", got, cut)
	}
}

// Writers and Readers that are never closed (the reference has no Close) give their device
// memory back when collected: 256 handles with 4 MiB rings would hold 1 GiB of HBM otherwise.
func TestHandlesFreedWithoutClose(t *testing.T) {
	p := bytes.Repeat([]byte("ts=3 level=info msg=\"ok\" "), 160)
	for k := 0; k < 256; k++ {
		var buf bytes.Buffer
		w := NewWriter(&buf, 4*MiB, 4096)
		if _, err := w.Write(p); err != nil {
			t.Fatal(err)
		}
		r := NewReaderBytes(buf.Bytes())
		q := make([]byte, len(p))
		if n, err := io.ReadFull(r, q); err != nil || n != len(p) || !bytes.Equal(q, p) {
			t.Fatalf("round trip %d: %v", k, err)
		}
		if k%32 == 31 {
			runtime.GC()
		}
	}
}
