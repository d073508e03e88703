// SBR / PS extension payloads of the host bitstream front end (include/jaad_parse.h).
#include "jaad_parse_internal.h"

namespace jaad {
namespace parse {

int parse_sbr(BitReader&, const Cfg&, bool, ParseState&, jaad_sbr_frame&) { return JAAD_ERR_UNSUPPORTED; }

int sbr_missing(const Cfg&, ParseState&, jaad_sbr_frame&) { return JAAD_ERR_UNSUPPORTED; }

}  // namespace parse
}  // namespace jaad
