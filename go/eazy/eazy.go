// Package eazy is the cgo drop-in for tlog-dev/eazy backed by the MI355X
// C-ABI (include/eazy.h, libeazy_amd.so).  It re-declares the reference
// package's exported identifiers with the same semantics: NewWriter /
// NewReader over io.Writer / io.Reader (writer.go:133, reader.go:79), the
// Writer / Reader fields, the error values (reader.go:57-76) and panics
// (writer.go:162-168), plus CompressBatch for many independent streams,
// which is where the GPU pays off.
//
// NOT COMPILED IN THIS REPOSITORY'S CI: the build image has no Go toolchain.
// The C++ host side (eazy_amd/cpp/eazy.hpp) implements the same logic and is
// what the tests exercise; this file is the binding a Go maintainer adds.
package eazy

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../eazy_amd -leazy_amd -Wl,-rpath,${SRCDIR}/../../eazy_amd
#include <stdlib.h>
#include "eazy.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"io"
	"runtime"
	"unsafe"
)

const (
	KiB = 1 << 10
	MiB = 1 << 20
)

// Token constants (writer.go:49-122).
const (
	Literal = C.EZ_LITERAL
	Copy    = C.EZ_COPY
	Meta    = C.EZ_META

	Len1   = C.EZ_LEN1
	Len2   = C.EZ_LEN2
	Len4   = C.EZ_LEN4
	LenAlt = C.EZ_LEN_ALT

	Off1    = C.EZ_OFF1
	Off2    = C.EZ_OFF2
	Off4    = C.EZ_OFF4
	OffLong = C.EZ_OFF_LONG

	MetaMagic = C.EZ_META_MAGIC
	MetaVer   = C.EZ_META_VER
	MetaReset = C.EZ_META_RESET
	MetaBreak = C.EZ_META_BREAK

	MetaLenWide = C.EZ_META_LEN_WIDE
	MetaLen0    = C.EZ_META_LEN0
	MetaTagMask = 0xf8
)

const Magic = "eazy"

// Errors (reader.go:57-76): the reference's values, text included.
var (
	ErrBadMagic           = errors.New("bad magic")
	ErrBlockSizeOverLimit = errors.New("block size is more than the limit")
	ErrNoMagic            = errors.New("no magic")
	ErrOverflow           = errors.New("length/offset overflow")
	ErrShortBuffer        = io.ErrShortBuffer
	ErrUnsupportedMeta    = errors.New("unsupported meta tag")
	ErrUnsupportedVersion = errors.New("unsupported file format version")
	ErrBreak              = errors.New("break point")
	ErrDevice             = errors.New("eazy: no usable MI355X")
)

// toErr maps a C-ABI status to the Go value the reference returns.  detail is
// the version (EZ_EUNSUPVER) or the meta id (EZ_EUNSUPMETA).  EZ_EINVAL is
// a reference panic; panicValue gives its value (callers know which it is).
func toErr(st C.int, detail int64) error {
	switch st {
	case C.EZ_OK:
		return nil
	case C.EZ_EOF:
		return io.EOF
	case C.EZ_ESHORTBUF:
		return ErrShortBuffer
	case C.EZ_EUNEXPECTEDEOF:
		return io.ErrUnexpectedEOF
	case C.EZ_EOVERFLOW:
		return ErrOverflow
	case C.EZ_EBADMAGIC:
		return ErrBadMagic
	case C.EZ_ENOMAGIC:
		return ErrNoMagic
	case C.EZ_EBLOCKLIMIT:
		return ErrBlockSizeOverLimit
	case C.EZ_EUNSUPMETA:
		return fmt.Errorf("%w: 0x%x", ErrUnsupportedMeta, detail) // reader.go:319
	case C.EZ_EUNSUPVER:
		return fmt.Errorf("%w: %v", ErrUnsupportedVersion, int(detail)) // reader.go:303
	case C.EZ_EBREAK:
		return ErrBreak
	case C.EZ_EMISSEDMETA:
		return errors.New("missed meta") // reader.go:155: a fresh value each time, as in Go
	case C.EZ_EINVAL:
		panic(panicValue(C.EZ_PANIC_OFFSET, 0))
	case C.EZ_EDEVICE:
		return ErrDevice
	}
	return fmt.Errorf("eazy: %s", C.GoString(C.ez_strerror(st)))
}

// panicValue is the value the reference panics with (writer.go:163, 167, 309,
// 562, 596): a string, or for Encoder.Meta the meta int itself (:601).
func panicValue(p C.int, meta int) interface{} {
	if p == C.EZ_PANIC_META {
		return meta
	}
	return C.GoString(C.ez_panic_message(p))
}

// sizePanic panics as Writer.init does on invalid sizes (writer.go:161-169).
func sizePanic(block, htable int) {
	if p := C.ez_writer_size_panic(C.int64_t(block), C.int64_t(htable)); p != C.EZ_PANIC_NONE {
		panic(panicValue(p, 0))
	}
}

func ptr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// Writer is the compressor (writer.go:17-46).  Not safe for concurrent use.
type Writer struct {
	Writer io.Writer

	// AppendMagic writes the magic before the first Write (default true).
	AppendMagic bool

	// FlushThreshold: 0 = flush every Write, -1 = manual Flush, N = flush
	// once N bytes are buffered (writer.go:27-34).
	FlushThreshold int

	h       *C.ez_writer
	b       []byte
	written int64
	resets  uint64 // stream restarts (WriteBatch's replay)
	ver     int
}

// Device is the HIP device NewWriter and NewReader put their handles on (no
// reference counterpart: the reference runs on the host).  Set it before
// creating handles, or use NewWriterOn / NewReaderOn.
var Device = 0

// NewWriter creates a new Writer (writer.go:133-145).  block and htable are
// powers of two; block is the window size, htable the hash table entries.
func NewWriter(wr io.Writer, block, htable int) *Writer {
	return NewWriterOn(wr, block, htable, Device)
}

// NewWriterOn is NewWriter with the handle on HIP device dev.
func NewWriterOn(wr io.Writer, block, htable, dev int) *Writer {
	sizePanic(block, htable)
	w := &Writer{Writer: wr, AppendMagic: true}
	if st := C.ez_writer_new(C.int64_t(block), C.int64_t(htable), C.int(dev), &w.h); st != C.EZ_OK {
		panic(toErr(st, 0))
	}
	// The reference Writer has nothing to release, so drop-in callers never Close:
	// the handle's device ring, table, HIP stream and pinned buffer go with the Writer.
	runtime.SetFinalizer(w, (*Writer).Close)
	return w
}

// Close releases the device state now (the reference has nothing to release; a
// Writer that is never closed releases it when it is garbage collected).
func (w *Writer) Close() {
	if w.h != nil {
		C.ez_writer_free(w.h)
		w.h = nil
	}
	runtime.SetFinalizer(w, nil)
}

func (w *Writer) sync() {
	m := 0
	if w.AppendMagic {
		m = 1
	}
	C.ez_writer_set_append_magic(w.h, C.int(m))
	C.ez_writer_set_version(w.h, C.int(w.ver))
}

// Write compresses p (writer.go:206-337).
func (w *Writer) Write(p []byte) (int, error) {
	w.sync()
	at := len(w.b)
	need := int(C.ez_compress_bound(C.size_t(len(p))))
	if cap(w.b)-at < need {
		nb := make([]byte, at, at+need)
		copy(nb, w.b)
		w.b = nb
	}
	out := w.b[at : at+need]
	var n C.size_t
	st := C.ez_writer_write(w.h, ptr(p), C.size_t(len(p)), ptr(out), C.size_t(need), &n)
	runtime.KeepAlive(w)
	if st != C.EZ_OK {
		return 0, w.failed(st)
	}
	w.b = w.b[:at+int(n)]
	if err := w.write(); err != nil {
		return 0, err
	}
	return len(p), nil
}

func (w *Writer) appendCall(f func(out *C.uint8_t, n C.size_t, got *C.size_t) C.int) error {
	w.sync()
	var tmp [32]byte
	var n C.size_t
	if st := f((*C.uint8_t)(unsafe.Pointer(&tmp[0])), 32, &n); st != C.EZ_OK {
		return toErr(st, 0)
	}
	w.b = append(w.b, tmp[:n]...)
	return w.write()
}

// WriteHeader writes the header if nothing was written yet (writer.go:342-350).
func (w *Writer) WriteHeader() error {
	if !w.isreset() {
		return nil
	}
	return w.appendCall(func(o *C.uint8_t, c C.size_t, n *C.size_t) C.int { return C.ez_writer_header(w.h, o, c, n) })
}

// WriteBreak writes the Break marker (writer.go:358-366).
func (w *Writer) WriteBreak() error {
	return w.appendCall(func(o *C.uint8_t, c C.size_t, n *C.size_t) C.int { return C.ez_writer_break(w.h, o, c, n) })
}

// Flush flushes the internal buffer (writer.go:371-377).
func (w *Writer) Flush() error {
	if len(w.b) == 0 {
		return nil
	}
	return w.flush()
}

// Reset restarts the stream on wr (writer.go:149-152).
func (w *Writer) Reset(wr io.Writer) { w.Writer = wr; w.reset() }

// ResetSize restarts the stream with new sizes (writer.go:155-159).
func (w *Writer) ResetSize(wr io.Writer, block, htable int) {
	w.Writer = wr
	sizePanic(block, htable)
	if st := C.ez_writer_reset_size(w.h, C.int64_t(block), C.int64_t(htable)); st != C.EZ_OK {
		panic(toErr(st, 0))
	}
	w.b = w.b[:0]
	w.written = 0
}

func (w *Writer) reset() { w.resets++; C.ez_writer_reset(w.h); w.b = w.b[:0]; w.written = 0 }

// failed: when the device history had taken the Write, the handle restarted its stream
// (it is reset now) and the mirror forgets w.b and written with it; a failure found before
// anything reached the device (no space, bad Write ends, no device) leaves both as they were.
// An EZ_EINVAL with a reference panic behind it re-panics with that value.
func (w *Writer) failed(st C.int) error {
	if C.ez_writer_is_reset(w.h) != 0 {
		w.resets++
		w.b = w.b[:0]
		w.written = 0
	}
	if st == C.EZ_EINVAL {
		if p := C.ez_writer_last_panic(w.h); p != C.EZ_PANIC_NONE {
			panic(panicValue(p, 0))
		}
		return errors.New("eazy: invalid Write arguments")
	}
	return toErr(st, 0)
}

// WriteBatch compresses several Writes in one device call (no reference counterpart): the sink
// sees what calling Write on each in turn gives it -- the handle reports where each Write's
// bytes end and FlushThreshold is replayed per Write; a short sink write that restarts the
// stream sends the remaining Writes through Write.  Returns the bytes of the Writes done.
func (w *Writer) WriteBatch(ps [][]byte) (int, error) {
	if len(ps) == 0 {
		return 0, nil
	}
	w.sync()
	var data []byte
	ends := make([]uint64, len(ps))
	need := 0
	for j, p := range ps {
		data = append(data, p...)
		ends[j] = uint64(len(data))
		need += int(C.ez_compress_bound(C.size_t(len(p))))
	}
	out := make([]byte, need+1)
	oe := make([]uint64, len(ps))
	st := C.ez_writer_write_batch(w.h, ptr(data), (*C.uint64_t)(unsafe.Pointer(&ends[0])), C.size_t(len(ps)),
		ptr(out), C.size_t(need), (*C.uint64_t)(unsafe.Pointer(&oe[0])))
	runtime.KeepAlive(w)
	if st != C.EZ_OK {
		return 0, w.failed(st)
	}
	gen, prev, done := w.resets, uint64(0), 0
	for j := range ps {
		w.b = append(w.b, out[prev:oe[j]]...)
		prev = oe[j]
		if err := w.write(); err != nil {
			return done, err
		}
		done += len(ps[j])
		if w.resets != gen { // the stream restarted: the rest on the new stream
			for _, p := range ps[j+1:] {
				n, err := w.Write(p)
				done += n
				if err != nil {
					return done, err
				}
			}
			break
		}
	}
	return done, nil
}

func (w *Writer) isreset() bool { return int(w.written)+len(w.b) == 0 }

func (w *Writer) write() error { // writer.go:379-385
	if w.FlushThreshold < 0 || len(w.b) < w.FlushThreshold {
		return nil
	}
	return w.flush()
}

func (w *Writer) flush() error { // writer.go:387-401
	n, err := w.Writer.Write(w.b)
	w.written += int64(n)
	if err != nil || n != len(w.b) {
		w.reset()
	}
	if err != nil {
		return err
	}
	w.b = w.b[:0]
	return nil
}

// Reader is the decompressor (reader.go:17-40).
type Reader struct {
	Reader io.Reader

	BlockSizeLimit      int
	BufferSize          int
	RequireMagic        bool
	SkipUnsupportedMeta bool

	h    *C.ez_reader
	b    []byte
	i    int
	boff int64
}

// NewReader creates a Reader over rd (reader.go:79-86).
func NewReader(rd io.Reader) *Reader { return NewReaderOn(rd, Device) }

// NewReaderOn is NewReader with the handle on HIP device dev.
func NewReaderOn(rd io.Reader, dev int) *Reader {
	r := &Reader{Reader: rd, BlockSizeLimit: 16 * MiB, BufferSize: 64 * KiB}
	r.open(dev)
	return r
}

// NewReaderBytes creates a Reader over b (reader.go:89-94).
func NewReaderBytes(b []byte) *Reader {
	r := &Reader{}
	r.open(Device)
	r.ResetBytes(b)
	return r
}

func (r *Reader) open(dev int) {
	if st := C.ez_reader_new(C.int(dev), &r.h); st != C.EZ_OK {
		panic(toErr(st, 0))
	}
	// as for Writer: drop-in callers never Close, the handle goes with the Reader
	runtime.SetFinalizer(r, (*Reader).Close)
}

// Close releases the device state now (a Reader that is never closed releases it
// when it is garbage collected).
func (r *Reader) Close() {
	if r.h != nil {
		C.ez_reader_free(r.h)
		r.h = nil
	}
	runtime.SetFinalizer(r, nil)
}

// Reset restarts decoding from rd (reader.go:96-99).
func (r *Reader) Reset(rd io.Reader) {
	r.ResetBytes(nil)
	r.Reader = rd
	C.ez_reader_set_whole(r.h, 0)
	runtime.KeepAlive(r)
}

// ResetBytes restarts decoding from b (reader.go:102-113).  b is the whole stream: the handle
// decodes it at once on the first Read and serves the Reads from that (ez_reader_set_whole).
func (r *Reader) ResetBytes(b []byte) {
	r.Reader = nil
	r.b = b
	r.i = 0
	r.boff = 0
	C.ez_reader_reset(r.h)
	C.ez_reader_set_whole(r.h, 1)
	runtime.KeepAlive(r)
}

// Read decompresses into p (reader.go:116-141).
func (r *Reader) Read(p []byte) (n int, err error) {
	magic, skip := 0, 0
	if r.RequireMagic {
		magic = 1
	}
	if r.SkipUnsupportedMeta {
		skip = 1
	}
	C.ez_reader_configure(r.h, C.int64_t(r.BlockSizeLimit), C.int(magic), C.int(skip))
	for n < len(p) && err == nil {
		var m, i C.size_t
		var det C.int64_t
		st := C.ez_reader_read(r.h, ptr(r.b), C.size_t(len(r.b)), C.size_t(r.i), C.int64_t(r.boff),
			ptr(p[n:]), C.size_t(len(p)-n), &m, &i, &det)
		runtime.KeepAlive(r)
		n += int(m)
		r.i = int(i)
		if n == len(p) {
			break
		}
		if st != C.EZ_ESHORTBUF {
			err = toErr(st, int64(det))
			continue
		}
		err = r.more()
		if errors.Is(err, io.EOF) && (C.ez_reader_pending(r.h) != 0 || r.i < len(r.b)) {
			err = io.ErrUnexpectedEOF
		}
	}
	return n, err
}

func (r *Reader) more() error { // reader.go:516-543
	if r.Reader == nil {
		return io.EOF
	}
	end := copy(r.b, r.b[r.i:])
	r.b = r.b[:end]
	r.boff += int64(r.i)
	r.i = 0
	if len(r.b) == 0 {
		r.b = make([]byte, r.BufferSize)
	} else {
		r.b = append(r.b, make([]byte, 1024)...)
	}
	r.b = r.b[:cap(r.b)]
	n, err := r.Reader.Read(r.b[end:])
	r.b = r.b[:end+n]
	if n != 0 && errors.Is(err, io.EOF) {
		err = nil
	}
	return err
}

// Devices lists the GPUs CompressBatch splits its batches over (contiguous whole-stream shards,
// one per entry; an entry may repeat); empty: every visible device.
var Devices []int

// CompressBatch compresses independent streams on the GPUs: the result for
// bufs[k] equals NewWriter(&buf, block, htable).Write(bufs[k]) into a fresh
// buffer.  The batch is sharded over Devices (every GPU by default); see INTEGRATION.md.
func CompressBatch(bufs [][]byte, block, htable int) ([][]byte, error) {
	return compressBatch(bufs, block, htable) // batch.go
}

// CompressStreams is the multi-Write batch (Go-only extension): stream k is a
// fresh NewWriter(block, htable) receiving streams[k][0], streams[k][1], ...
// through Write with FlushThreshold 0; the result is what its sink receives.
// Streams with 2 x total length > block are refused (EINVAL).
func CompressStreams(streams [][][]byte, block, htable int) ([][]byte, error) {
	return compressStreams(streams, block, htable) // batch.go
}
