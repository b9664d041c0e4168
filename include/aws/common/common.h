#pragma once
/*
 * Minimal aws-c-common surface needed by the Aws::Crt::Checksum drop-in and its tests
 * (tests/CRCTest.cpp, tests/XXHashTest.cpp of the reference).  aws-c-common itself is an
 * un-vendored submodule of the reference (.gitmodules:1-4); this shim provides only the byte
 * cursor / byte buffer / allocator / error pieces the checksum path touches.  In a full CRT build
 * these symbols come from the real aws-c-common instead.
 */
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <aws/common/allocator.h>
#include <aws/common/byte_buf.h>
#include <aws/common/error.h>
