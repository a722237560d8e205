/* Legacy helper functions (include/convHelpers.h; reference src/convHelpers.c:3-14). */
#include "convHelpers.h"

void unpackBigToLittleEndian(uint8_t* unpackArray, int unpackArrayLen, uint64_t packed) {
    for (int i = 0; i < unpackArrayLen; i++) unpackArray[i] = (uint8_t)((packed >> (unpackArrayLen - 1 - i)) & 1u);
}

void unpackLittleToLittleEndian(uint8_t* unpackArray, int unpackArrayLen, uint64_t packed) {
    for (int i = 0; i < unpackArrayLen; i++) unpackArray[i] = (uint8_t)((packed >> i) & 1u);
}
