/*
 * sddc_compat/r2iq.h
 *
 * Used only for builds of this repository WITHOUT the ExtIO_sddc tree (the tests, the GPU
 * box).  In the integration build the tree's Core/r2iq.h comes first on the include path
 * and this file is not seen.
 *
 * What it must preserve: the object layout and vtable of the boundary base class described
 * in SURVEY.md §8(b) (Core/r2iq.h:16-48), so a caller compiled against either header talks
 * to the same object.  Itanium x86-64 layout, checked by static_asserts in
 * extio_sddc_amd/csrc/r2iq/fft_mt_r2iq.cpp and by the byte probe in tests/harness:
 *
 *     offset  0  vptr
 *     offset  8  int   decimation index
 *     offset 12  bool  running flag
 *     offset 16  int   ratio table [7]
 *     offset 44  bool  RAND de-randomisation
 *     offset 45  bool  lower-sideband conjugation          sizeof = 48
 *
 * Virtual slots, in order: destructor (complete, deleting), Init, TurnOn, TurnOff, IsOn,
 * DataReady, setFreqOffset.  The small setters and getters are non-virtual inlines, so they
 * compile into the caller and only touch the fields above.
 */
#ifndef R2IQ_H
#define R2IQ_H

#define NDECIDX 7 /* decimation indices 0..6 */

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "dsp/ringbuffer.h"

struct r2iqThreadArg;

class r2iqControlClass
{
public:
    r2iqControlClass(); // out of line, supplied by the DDC (extio_sddc_amd/csrc/r2iq/fft_mt_r2iq.cpp)
    virtual ~r2iqControlClass() {}

    // -- inline field accessors (caller-side code) --
    int getRatio() { return mratio[mdecimation]; }
    void updateRand(bool on) { randADC = on; }
    bool getRand() const { return randADC; }
    void setSideband(bool lower) { sideband = lower; }
    bool getSideband() const { return sideband; }
    void setDecimate(int index) { mdecimation = index; }

    // -- virtual interface (slot order fixed by the ABI) --
    virtual void Init(float gainScale, ringbuffer<int16_t> *samplesIn, ringbuffer<float> *iqOut) {}
    virtual void TurnOn() { r2iqOn = true; }
    virtual void TurnOff(void) { r2iqOn = false; }
    virtual bool IsOn(void) { return r2iqOn; }
    virtual void DataReady(void) {}
    virtual float setFreqOffset(float fractionOfHalfRate) { return 0; }

protected:
    int mdecimation;     // output rate = ADC rate / 2^(index + 1)
    bool r2iqOn;         // set by TurnOn, cleared by TurnOff
    int mratio[NDECIDX]; // 1, 2, 4, ... 64

private:
    bool randADC;        // odd samples arrive XORed with 0xFFFE
    bool sideband;       // conjugate the output
};

#endif /* R2IQ_H */
