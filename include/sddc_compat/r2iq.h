/*
 * sddc_compat/r2iq.h — standalone stand-in for the ExtIO_sddc boundary class, used ONLY
 * when this repository is built without the ExtIO_sddc tree (tests, the GPU box).
 *
 * In the integration build the reference's own Core/r2iq.h is first on
 * the include path and this file is never seen.  It restates the interface of
 * r2iqControlClass (Core/r2iq.h:16-48) with an identical object layout, so code
 * compiled against either header is ABI-compatible (x86-64 Itanium ABI: vptr @0,
 * mdecimation @8, r2iqOn @12, mratio[7] @16, randADC @44, sideband @45, sizeof 48;
 * checked by static_asserts in extio_sddc_amd/csrc/r2iq/fft_mt_r2iq.cpp).
 */
#ifndef R2IQ_H
#define R2IQ_H

#define NDECIDX 7  /* number of decimation ratios, r2iq.h:5 */

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "dsp/ringbuffer.h"

struct r2iqThreadArg;

class r2iqControlClass {
public:
    r2iqControlClass();                 /* defined by the DDC implementation (fft_mt_r2iq.cpp) */
    virtual ~r2iqControlClass() {}

    /* non-virtual accessors, inlined into callers such as RadioHandler */
    int getRatio() { return mratio[mdecimation]; }
    void updateRand(bool v) { randADC = v; }
    bool getRand() const { return randADC; }
    void setSideband(bool lsb) { sideband = lsb; }
    bool getSideband() const { return sideband; }
    void setDecimate(int dec) { mdecimation = dec; }

    /* virtual interface, vtable order as in the reference */
    virtual void Init(float gain, ringbuffer<int16_t> *input, ringbuffer<float> *obuffers) {}
    virtual void TurnOn() { r2iqOn = true; }
    virtual void TurnOff(void) { r2iqOn = false; }
    virtual bool IsOn(void) { return r2iqOn; }
    virtual void DataReady(void) {}
    virtual float setFreqOffset(float offset) { return 0; }

protected:
    int mdecimation;        /* 0..6: output rate = ADC rate / 2^(d+1) */
    bool r2iqOn;
    int mratio[NDECIDX];    /* 2^d */

private:
    bool randADC;           /* ADC RAND mode: de-randomise on conversion */
    bool sideband;          /* true: conjugate the IQ (lower sideband) */
};

#endif
