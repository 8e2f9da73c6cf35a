// The shared-memory ring primitives (csrc/core/shmring.cpp) compiled into the
// device-runtime module too: _hip and _core are separate extension modules with
// hidden symbols, and the DeviceServer (here) creates the segments that the
// control plane's same-node connections (there) attach to.
#include "shmring.cpp"
