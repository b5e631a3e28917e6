package eazy

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#include <stdint.h>
#include "eazy.h"
#include <hip/hip_runtime_api.h>
#cgo LDFLAGS: -L/opt/rocm/lib -lamdhip64
*/
import "C"

import (
	"errors"
	"unsafe"
)

// compressBatch: one stream per buffer (one Write each), through ez_compress_batch_multi: the
// batch is split into contiguous whole-stream shards over every visible device (Devices, when set),
// one host thread and HIP stream per device, and the packed result comes back in host memory.
func compressBatch(bufs [][]byte, block, htable int) ([][]byte, error) {
	sizePanic(block, htable) // Writer.init writer.go:161-169, as NewWriter would
	count := len(bufs)
	if count == 0 {
		return nil, nil
	}
	inOff := make([]uint64, count+1)
	capacity := uint64(16)
	for k, b := range bufs {
		inOff[k+1] = inOff[k] + uint64(len(b))
		capacity += uint64(C.ez_compress_bound(C.size_t(len(b))))
	}
	host := make([]byte, 0, inOff[count]+1)
	for _, b := range bufs {
		host = append(host, b...)
	}
	host = append(host, 0) // (a valid pointer for an all-empty batch)
	packed := make([]byte, capacity)
	packedOff := make([]uint64, count+1)
	status := make([]int32, count)
	var devs *C.int
	ndev := 0
	if len(Devices) > 0 {
		cd := make([]C.int, len(Devices))
		for k, d := range Devices {
			cd[k] = C.int(d)
		}
		devs, ndev = &cd[0], len(cd)
	}
	st := C.ez_compress_batch_multi(C.int64_t(block), C.int64_t(htable), 0, (*C.uint8_t)(unsafe.Pointer(&host[0])),
		(*C.uint64_t)(unsafe.Pointer(&inOff[0])), C.uint64_t(count), devs, C.int(ndev), (*C.uint8_t)(unsafe.Pointer(&packed[0])),
		C.uint64_t(capacity), (*C.uint64_t)(unsafe.Pointer(&packedOff[0])), (*C.int32_t)(unsafe.Pointer(&status[0])))
	if st != C.EZ_OK {
		return nil, toErr(st, 0)
	}
	res := make([][]byte, count)
	for k := range bufs {
		if status[k] != 0 {
			return nil, errors.Join(ErrDevice, toErr(C.int(status[k]), 0))
		}
		res[k] = packed[packedOff[k]:packedOff[k+1]:packedOff[k+1]]
	}
	return res, nil
}

// compressStreams stages the streams into device memory, runs K1 (stream k =
// NewWriter(block, htable) receiving the Writes streams[k] in order,
// FlushThreshold 0) and copies every slot back.  One HIP stream per call.
func compressStreams(streams [][][]byte, block, htable int) ([][]byte, error) {
	sizePanic(block, htable) // Writer.init writer.go:161-169, as NewWriter would
	count := len(streams)
	if count == 0 {
		return nil, nil
	}
	inOff := make([]uint64, count+1)
	outOff := make([]uint64, count+1)
	writeIdx := make([]uint64, count+1)
	var writeEnd []uint64
	maxLen, maxWrites, multi := 0, 1, false
	for k, ws := range streams {
		n := 0
		for _, w := range ws {
			n += len(w)
			writeEnd = append(writeEnd, inOff[k]+uint64(n))
		}
		if len(ws) != 1 {
			multi = true
		}
		if len(ws) > maxWrites {
			maxWrites = len(ws)
		}
		inOff[k+1] = inOff[k] + uint64(n)
		writeIdx[k+1] = uint64(len(writeEnd))
		outOff[k+1] = outOff[k] + uint64(C.ez_compress_bound(C.size_t(n))) + 5*uint64(len(ws))
		if n > maxLen {
			maxLen = n
		}
	}
	host := make([]byte, 0, inOff[count])
	for _, ws := range streams {
		for _, w := range ws {
			host = append(host, w...)
		}
	}
	var dIn, dOut, dInOff, dOutOff, dSize, dStatus, dWIdx, dWEnd unsafe.Pointer
	alloc := func(p *unsafe.Pointer, n uint64) error {
		if C.hipMalloc(p, C.size_t(n+16)) != C.hipSuccess {
			return ErrDevice
		}
		return nil
	}
	defer func() {
		for _, p := range []unsafe.Pointer{dIn, dOut, dInOff, dOutOff, dSize, dStatus, dWIdx, dWEnd} {
			if p != nil {
				C.hipFree(p)
			}
		}
	}()
	// every HIP call's result is checked: a failed copy must never hand back stale bytes as success
	// (the errors surface as the reference's do, writer.go:387-401)
	hip := func(r C.hipError_t) error {
		if r != C.hipSuccess {
			return ErrDevice
		}
		return nil
	}
	for _, a := range []struct {
		p *unsafe.Pointer
		n uint64
	}{{&dIn, inOff[count]}, {&dOut, outOff[count]}, {&dInOff, 8 * uint64(count+1)}, {&dOutOff, 8 * uint64(count+1)},
		{&dSize, 8 * uint64(count)}, {&dStatus, 4 * uint64(count)}, {&dWIdx, 8 * uint64(count+1)},
		{&dWEnd, 8 * uint64(len(writeEnd))}} {
		if err := alloc(a.p, a.n); err != nil {
			return nil, err
		}
	}
	if len(host) > 0 {
		if err := hip(C.hipMemcpy(dIn, unsafe.Pointer(&host[0]), C.size_t(len(host)), C.hipMemcpyHostToDevice)); err != nil {
			return nil, err
		}
	}
	if err := hip(C.hipMemcpy(dInOff, unsafe.Pointer(&inOff[0]), C.size_t(8*(count+1)), C.hipMemcpyHostToDevice)); err != nil {
		return nil, err
	}
	if err := hip(C.hipMemcpy(dOutOff, unsafe.Pointer(&outOff[0]), C.size_t(8*(count+1)), C.hipMemcpyHostToDevice)); err != nil {
		return nil, err
	}
	b := C.ez_batch{
		in: (*C.uint8_t)(dIn), in_off: (*C.uint64_t)(dInOff), out: (*C.uint8_t)(dOut), out_off: (*C.uint64_t)(dOutOff),
		out_size: (*C.uint64_t)(dSize), status: (*C.int32_t)(dStatus), count: C.uint64_t(count), max_len: C.uint64_t(maxLen),
	}
	var st C.int
	if multi {
		if err := hip(C.hipMemcpy(dWIdx, unsafe.Pointer(&writeIdx[0]), C.size_t(8*(count+1)), C.hipMemcpyHostToDevice)); err != nil {
			return nil, err
		}
		if len(writeEnd) > 0 {
			if err := hip(C.hipMemcpy(dWEnd, unsafe.Pointer(&writeEnd[0]), C.size_t(8*len(writeEnd)), C.hipMemcpyHostToDevice)); err != nil {
				return nil, err
			}
		}
		st = C.ez_compress_batch_writes(C.int64_t(block), C.int64_t(htable), 0, &b, (*C.uint64_t)(dWIdx),
			(*C.uint64_t)(dWEnd), C.uint64_t(maxWrites), nil)
	} else {
		st = C.ez_compress_batch(C.int64_t(block), C.int64_t(htable), 0, &b, nil)
	}
	if st != C.EZ_OK {
		return nil, toErr(st, 0)
	}
	out := make([]byte, outOff[count])
	size := make([]uint64, count)
	status := make([]int32, count)
	// (hipMemcpy to host waits for the batch's kernels on the null stream, and reports their faults)
	if err := hip(C.hipMemcpy(unsafe.Pointer(&out[0]), dOut, C.size_t(len(out)), C.hipMemcpyDeviceToHost)); err != nil {
		return nil, err
	}
	if err := hip(C.hipMemcpy(unsafe.Pointer(&size[0]), dSize, C.size_t(8*count), C.hipMemcpyDeviceToHost)); err != nil {
		return nil, err
	}
	if err := hip(C.hipMemcpy(unsafe.Pointer(&status[0]), dStatus, C.size_t(4*count), C.hipMemcpyDeviceToHost)); err != nil {
		return nil, err
	}
	res := make([][]byte, count)
	for k := range streams {
		if status[k] != 0 {
			return nil, errors.Join(ErrDevice, toErr(C.int(status[k]), 0))
		}
		res[k] = out[outOff[k] : outOff[k]+size[k]]
	}
	return res, nil
}
