/* TEST INFRASTRUCTURE: embeds the oracle's v_rcp_f32 model table (build/rcp_codes.bin, unpacked
   from rcp_gfx950.bin.xz by the Makefile; see make_rcp_table.py) as o_rcp_codes[2^21]. */
        .section .rodata
        .global o_rcp_codes
        .type o_rcp_codes, @object
        .balign 64
o_rcp_codes:
        .incbin RCP_CODES_BIN
        .size o_rcp_codes, . - o_rcp_codes
        .section .note.GNU-stack, "", @progbits
