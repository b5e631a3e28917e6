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

// compressBatch stages the buffers into device memory, runs K1 (one stream
// per buffer) and copies every slot back.  One HIP stream per call.
func compressBatch(bufs [][]byte, block, htable int) ([][]byte, error) {
	count := len(bufs)
	if count == 0 {
		return nil, nil
	}
	inOff := make([]uint64, count+1)
	outOff := make([]uint64, count+1)
	maxLen := 0
	for k, b := range bufs {
		inOff[k+1] = inOff[k] + uint64(len(b))
		outOff[k+1] = outOff[k] + uint64(C.ez_compress_bound(C.size_t(len(b))))
		if len(b) > maxLen {
			maxLen = len(b)
		}
	}
	host := make([]byte, 0, inOff[count])
	for _, b := range bufs {
		host = append(host, b...)
	}
	var dIn, dOut, dInOff, dOutOff, dSize, dStatus unsafe.Pointer
	alloc := func(p *unsafe.Pointer, n uint64) error {
		if C.hipMalloc(p, C.size_t(n+16)) != C.hipSuccess {
			return ErrDevice
		}
		return nil
	}
	defer func() {
		for _, p := range []unsafe.Pointer{dIn, dOut, dInOff, dOutOff, dSize, dStatus} {
			if p != nil {
				C.hipFree(p)
			}
		}
	}()
	for _, a := range []struct {
		p *unsafe.Pointer
		n uint64
	}{{&dIn, inOff[count]}, {&dOut, outOff[count]}, {&dInOff, 8 * uint64(count+1)}, {&dOutOff, 8 * uint64(count+1)},
		{&dSize, 8 * uint64(count)}, {&dStatus, 4 * uint64(count)}} {
		if err := alloc(a.p, a.n); err != nil {
			return nil, err
		}
	}
	if len(host) > 0 {
		C.hipMemcpy(dIn, unsafe.Pointer(&host[0]), C.size_t(len(host)), C.hipMemcpyHostToDevice)
	}
	C.hipMemcpy(dInOff, unsafe.Pointer(&inOff[0]), C.size_t(8*(count+1)), C.hipMemcpyHostToDevice)
	C.hipMemcpy(dOutOff, unsafe.Pointer(&outOff[0]), C.size_t(8*(count+1)), C.hipMemcpyHostToDevice)
	b := C.ez_batch{
		in: (*C.uint8_t)(dIn), in_off: (*C.uint64_t)(dInOff), out: (*C.uint8_t)(dOut), out_off: (*C.uint64_t)(dOutOff),
		out_size: (*C.uint64_t)(dSize), status: (*C.int32_t)(dStatus), count: C.uint64_t(count), max_len: C.uint64_t(maxLen),
	}
	if st := C.ez_compress_batch(C.int64_t(block), C.int64_t(htable), 0, &b, nil); st != C.EZ_OK {
		return nil, toErr(st, 0)
	}
	out := make([]byte, outOff[count])
	size := make([]uint64, count)
	status := make([]int32, count)
	C.hipMemcpy(unsafe.Pointer(&out[0]), dOut, C.size_t(len(out)), C.hipMemcpyDeviceToHost)
	C.hipMemcpy(unsafe.Pointer(&size[0]), dSize, C.size_t(8*count), C.hipMemcpyDeviceToHost)
	C.hipMemcpy(unsafe.Pointer(&status[0]), dStatus, C.size_t(4*count), C.hipMemcpyDeviceToHost)
	res := make([][]byte, count)
	for k := range bufs {
		if status[k] != 0 {
			return nil, errors.Join(ErrDevice, toErr(C.int(status[k]), 0))
		}
		res[k] = out[outOff[k] : outOff[k]+size[k]]
	}
	return res, nil
}
