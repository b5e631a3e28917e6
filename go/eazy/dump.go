package eazy

// Dumper / NewDumper / Dump: the reference's debug printer of a compressed stream
// (reader.go:43-54 the type, :545-555 Dump, :557-561 NewDumper, :563-600 ReadFrom,
// :602-710 Write, :712-732 Close).  Host side, as in the reference: the tokens are
// walked with the C-ABI's Decoder (codec.go); no GPU is involved.  The printed text
// (Go fmt verbs) is part of the interface and is the reference's; the C++ mirror
// (eazy_amd/cpp/eazy.hpp Dump) and the Python one (eazy_amd/dump.py) print the same.
//
// NOT COMPILED IN THIS REPOSITORY'S CI (no Go toolchain in the image), like eazy.go.

import (
	"errors"
	"fmt"
	"io"
)

// Dumper prints one line per padding run, meta, literal and copy of the
// compressed bytes written to it (reader.go:43-54).
type Dumper struct {
	io.Writer

	// Debug, when set, is called once per printed item: input range [ioff, iend),
	// output offset, the item kind ('p', 'm', 'l', 'c', 'e'), its length and offset
	// (the meta id for 'm').
	Debug func(ioff, iend, ooff int64, tag byte, l, off int)

	// GlobalOffset < 0 drops the global-offset column.
	GlobalOffset int64

	dec  Decoder
	pos  int64 // output position of the next token (the reader's pos)
	boff int64 // input consumed by earlier Writes
	b    []byte
	p    []byte // ReadFrom's buffer
}

// NewDumper creates a Dumper printing to w (reader.go:557-561).
func NewDumper(w io.Writer) *Dumper { return &Dumper{Writer: w} }

// Dump is the debug print of a whole compressed buffer, with the error that
// stopped the walk appended (reader.go:545-555).
func Dump(p []byte) string {
	d := Dumper{}
	_, err := d.Write(p)
	_ = d.Close()
	text := d.b
	if err != nil {
		text = append(append(text, "\nerror: "...), err.Error()...)
	}
	return string(text)
}

func (d *Dumper) debug(st, i int, kind byte, l, off int) {
	if d.Debug != nil {
		d.Debug(d.boff+int64(st), d.boff+int64(i), d.pos, kind, l, off)
	}
}

// Write prints every whole token of p; it returns how many bytes those took
// (reader.go:602-710).  A token cut by the end of p stops the walk with
// ErrShortBuffer; ReadFrom keeps the rest for the next call.
func (d *Dumper) Write(p []byte) (done int, err error) {
	d.b = d.b[:0]
	defer d.flushLine(&done, &err)
	i := 0
	for i < len(p) {
		st := i
		if d.GlobalOffset >= 0 {
			d.b = fmt.Appendf(d.b, "%6x  ", d.GlobalOffset+int64(st))
		}
		d.b = fmt.Appendf(d.b, "%4x  %6x  ", st, d.pos)
		for i < len(p) && p[i] == 0 { // padding
			i++
		}
		if i > st {
			d.b = fmt.Appendf(d.b, "pad  %4x\n", i-st)
			d.debug(st, i, 'p', i-st, 0)
			done = i
			continue
		}
		tag, l, j, e := d.dec.Tag(p, i)
		if e != nil {
			return st, e
		}
		switch {
		case tag == Meta && l == 0:
			meta, ml, k, e := d.dec.Meta(p, j)
			if e != nil {
				return k, e
			}
			if k+ml > len(p) {
				return k, ErrShortBuffer
			}
			arg := p[k : k+ml]
			if meta == MetaVer && ml == 1 {
				d.dec.Ver = int(arg[0])
			}
			d.b = fmt.Appendf(d.b, "meta %2x %x  %-8q  % x\n", meta>>3, ml, arg, arg)
			d.debug(st, k, 'm', ml, meta)
			i = k + ml
		case tag == Literal:
			if j+l > len(p) {
				return j, ErrShortBuffer
			}
			d.b = fmt.Appendf(d.b, "lit  %4x        %q\n", l, p[j:j+l])
			d.debug(st, j, 'l', l, 0)
			i = j + l
			d.pos += int64(l)
		default: // Copy
			note := ""
			if j < len(p) && p[j] == OffLong {
				note = "  (long)"
			}
			off, k, e := d.dec.Offset(p, j, l)
			if e != nil {
				return st, e
			}
			d.b = fmt.Appendf(d.b, "copy %4x  off %4x%s\n", l, off, note)
			d.debug(st, k, 'c', l, off)
			i = k
			d.pos += int64(l)
		}
		done = i
	}
	return i, nil
}

// flushLine is Write's epilogue: account the consumed bytes and hand the text to
// the sink (its error only when the walk had none).
func (d *Dumper) flushLine(done *int, err *error) {
	d.boff += int64(*done)
	if d.GlobalOffset >= 0 {
		d.GlobalOffset += int64(*done)
	}
	if d.Writer == nil {
		return
	}
	if _, e := d.Writer.Write(d.b); *err == nil {
		*err = e
	}
}

// ReadFrom dumps everything r yields, carrying a token cut by a read boundary
// over to the next read (reader.go:563-600).
func (d *Dumper) ReadFrom(r io.Reader) (total int64, err error) {
	if d.p == nil {
		d.p = make([]byte, 0x10000)
	}
	kept := 0
	for {
		var n int
		n, err = r.Read(d.p[kept:])
		if n == 0 {
			break
		}
		total += int64(n)
		var used int
		used, err = d.Write(d.p[:kept+n])
		kept = copy(d.p, d.p[used:kept+n])
		if err != nil && !errors.Is(err, ErrShortBuffer) {
			break
		}
	}
	if errors.Is(err, io.EOF) {
		err = nil
	}
	if err == nil && kept != 0 {
		err = io.ErrUnexpectedEOF
	}
	return total, err
}

// Close prints the closing offsets line (reader.go:712-732).
func (d *Dumper) Close() error {
	if d.GlobalOffset >= 0 {
		d.b = fmt.Appendf(d.b, "%6x  ", d.GlobalOffset)
	}
	d.b = fmt.Appendf(d.b, "%4x  %6x  ", 0, d.pos)
	if d.Debug != nil {
		d.Debug(d.boff, d.boff, d.pos, 'e', 0, 0)
	}
	return nil
}
