// The fused sort + drain for the hash-probe and affine routes (modes 0 and 2): the
// same source as mailbox_sort_fused.hip, compiled as its own object.
#define PT_FUSED_OTHER_MODES 1
#include "mailbox_sort_fused.hip"
