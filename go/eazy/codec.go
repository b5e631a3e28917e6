package eazy

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#include "eazy.h"
*/
import "C"

import "unsafe"

// Encoder is the token encoder (writer.go:537-621) over the C-ABI's host codec.
type Encoder struct {
	Ver int
}

// Decoder is the token decoder (reader.go:346-514) over the C-ABI's host codec.
type Decoder struct {
	Ver int
}

func (e Encoder) app(b []byte, p C.int, meta int, f func(d *C.uint8_t, c C.size_t, n *C.size_t) C.int) []byte {
	var tmp [16]byte
	var n C.size_t
	if st := f((*C.uint8_t)(unsafe.Pointer(&tmp[0])), 16, &n); st != C.EZ_OK {
		if st == C.EZ_EINVAL {
			panic(panicValue(p, meta))
		}
		panic(toErr(st, 0))
	}
	return append(b, tmp[:n]...)
}

// Tag appends a literal/copy tag of length l (writer.go:537-563); panics "too big length".
func (e Encoder) Tag(b []byte, tag byte, l int) []byte {
	return e.app(b, C.EZ_PANIC_LENGTH, 0, func(d *C.uint8_t, c C.size_t, n *C.size_t) C.int {
		return C.ez_encode_tag(d, c, n, C.int(tag), C.int64_t(l))
	})
}

// Offset appends a copy offset (writer.go:565-597); panics "too big offset".
func (e Encoder) Offset(b []byte, off, l int) []byte {
	return e.app(b, C.EZ_PANIC_OFFSET, 0, func(d *C.uint8_t, c C.size_t, n *C.size_t) C.int {
		return C.ez_encode_offset(d, c, n, C.int64_t(off), C.int64_t(l))
	})
}

// Meta appends a meta tag (writer.go:599-621); panics with meta itself for a bad id.
func (e Encoder) Meta(b []byte, meta, l int) []byte {
	p := C.int(C.EZ_PANIC_OFFSET)
	if meta&^MetaTagMask != 0 {
		p = C.EZ_PANIC_META
	}
	return e.app(b, p, meta, func(d *C.uint8_t, c C.size_t, n *C.size_t) C.int {
		return C.ez_encode_meta(d, c, n, C.int64_t(meta), C.int64_t(l))
	})
}

// Tag decodes a tag at b[st:] (reader.go:346-392); i == st on error.
func (d Decoder) Tag(b []byte, st int) (tag, l, i int, err error) {
	var t C.int
	var ll C.int64_t
	var j C.size_t
	e := C.ez_decode_tag(ptr(b), C.size_t(len(b)), C.size_t(st), &t, &ll, &j)
	return int(t), int(ll), int(j), toErr(e, 0)
}

// Offset decodes a copy offset at b[st:] (reader.go:394-472).
func (d Decoder) Offset(b []byte, st, l int) (off, i int, err error) {
	var o C.int64_t
	var j C.size_t
	e := C.ez_decode_offset(ptr(b), C.size_t(len(b)), C.size_t(st), C.int64_t(l), &o, &j)
	return int(o), int(j), toErr(e, 0)
}

// Meta decodes a meta tag at b[st:] (reader.go:474-514).
func (d Decoder) Meta(b []byte, st int) (meta, l, i int, err error) {
	var m, ll C.int64_t
	var j C.size_t
	e := C.ez_decode_meta(ptr(b), C.size_t(len(b)), C.size_t(st), &m, &ll, &j)
	return int(m), int(ll), int(j), toErr(e, 0)
}

// status codes for tests (cgo identifiers cannot be used in _test.go files)
const (
	C_EUNSUPMETA = C.EZ_EUNSUPMETA
	C_EUNSUPVER  = C.EZ_EUNSUPVER
)
