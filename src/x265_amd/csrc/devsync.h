// devsync.h — HIP entries that synchronise the whole device (hipHostRegister / hipHostUnregister: measured,
// round 6) wait for every running kernel, a resident one too: the RDO server (X265AMD_RDO_SERVER,
// rdosession.cpp) would hold such a call until its lifetime ends.  Every such call in the library runs inside a
// DevSyncScope, which stops the resident servers first and keeps them from relaunching until it ends (their
// posted requests wait and are served by the next launch).
#pragma once

extern "C" void x265amd_devsync_begin(void);
extern "C" void x265amd_devsync_end(void);

struct DevSyncScope
{
    DevSyncScope() { x265amd_devsync_begin(); }
    ~DevSyncScope() { x265amd_devsync_end(); }
    DevSyncScope(const DevSyncScope&) = delete;
    DevSyncScope& operator=(const DevSyncScope&) = delete;
};
