/* gasal_header.h — umbrella header, drop-in for Non-CDP/GASAL2/src/gasal_header.h. */
#ifndef __GASAL_HEADER_H__
#define __GASAL_HEADER_H__

#include "gasal.h"
#include "args_parser.h"
#include "gasal_align.h"
#include "host_batch.h"
#include "ctors.h"
#include "interfaces.h"

#endif
