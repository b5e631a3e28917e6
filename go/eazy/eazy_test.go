package eazy

// A few of the reference's known answers (eazy_test.go), for a Go box with an
// MI355X: go test ./go/eazy

import (
	"bytes"
	"io"
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
	got, err := CompressBatch(bufs, MiB, 1024)
	if err != nil {
		t.Fatal(err)
	}
	for k, p := range bufs {
		var buf bytes.Buffer
		NewWriter(&buf, MiB, 1024).Write(p)
		if len(p) > 0 && !bytes.Equal(got[k], buf.Bytes()) {
			t.Fatalf("stream %d differs", k)
		}
	}
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
