// compat/rc4/rc4_encryption.h -- zero-edit drop-in for the reference's
// <rc4/rc4_encryption.h> (/root/reference/depends/rc4/rc4_encryption.h:43-99).
//
// Put  -I<repo>/include/compat -I<repo>/include  BEFORE the reference's
// -I depends  and every `#include <rc4/rc4_encryption.h>` of zsummerX
// (include/zsummerX/frame/session.h:43, include/zsummerX/common/common.h:78)
// resolves here: the global name RC4Encryption becomes the gfx950-backed
// mirror class, and src/frame/session.cpp compiles unchanged
// (tests/test_reference_binding.py compiles it).  Link with -lzrc4.
#pragma once
#include <zsummerx_amd/rc4_encryption.h>

using zsummerx_amd::RC4Encryption;
