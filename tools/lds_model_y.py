TMAP4 = [[64, 68, 72, 46, 65, 84, 24, 28, 32, 85, 25, 44, 48, 52, 26, 45],
    [49, 53, 27, 31, 50, 69, 88, 92, 66, 70, 89, 29, 33, 86, 90, 30],
    [98, 38, 57, 76, 99, 39, 58, 77, 96, 36, 59, 78, 97, 37, 56, 79],
    [0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15],
    [34, 87, 91, 95, 35, 54, 73, 47, 51, 55, 74, 93, 67, 71, 75, 94],
    [83, 23, 42, 61, 80, 20, 43, 62, 81, 21, 40, 63, 82, 22, 41, 60],
    [19, 117, 121, 125, 16, 118, 122, 126, 17, 119, 123, 127, 18, 116, 120, 124],
    [113, 102, 106, 110, 114, 103, 107, 111, 115, 100, 104, 108, 112, 101, 105, 109]]
PART_B=16896; BOARD_B=2*PART_B
def cell(b,r): return b*BOARD_B + 8192*(r>>4) + 16*((r+4*b)&15)
def zcell(wb):
    wb = wb if (wb & 2) else wb ^ 2
    r = 30 + (wb & 1)
    return cell(((wb - r) & 15) >> 2, r)
def entry(nvb, t, ln, tap):
    n, gg = ln & 15, ln >> 4
    v = TMAP4[t][n] if nvb == 4 else ((t & 3) | ((16*(t>>2)+n) << 2))
    b, p = v & 3, v >> 2
    dh, dw = tap//3-1, tap%3-1
    r, c, s = p//5+dh, p%5+dw, p+5*dh+dw
    valid = p < 30 and 0 <= r < 6 and 0 <= c < 5
    return (cell(b,s) if valid else zcell(s+4*b)) + 256*gg
G128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128 += [[l+32 for l in g] for g in G128]
def cycles(addrs):
    tot=0
    for g in G128:
        banks={}
        for l in g:
            a=addrs[l]
            for d in range(4):
                bk=(a//4+d)%64
                banks.setdefault(bk,set()).add(a//4+d)
        tot+=max(len(v) for v in banks.values())
    return tot
def act(t, tap):
    dr, dc = tap//3-1, tap%3-1
    return {0:True,1:True,2:dc!=1,3:dr!=-1,4:True,5:dc!=-1,6:dc!=1,7:dr!=1}[t]
for nvb in (4,3,2,1):
    tot=0; ideal=0
    for tap in range(9):
        for t in range(8):
            if nvb==4 and not act(t,tap): continue
            if nvb<4 and (t&3)>=nvb: continue
            for kb in range(8):
                for part in range(2):
                    addrs=[entry(nvb,t,l,tap)+1024*kb+part*PART_B for l in range(64)]
                    tot+=cycles(addrs); ideal+=4
    print(nvb, 'cycles', tot, 'ideal', ideal, 'extra frac', (tot-ideal)/tot)
print('--- per tap, nvb=1, tile 0 / 4, kb 0 part 0')
for tap in range(9):
    for t in (0,4):
        addrs=[entry(1,t,l,tap) for l in range(64)]
        res=[((a%256)//16) for a in addrs[:32]]
        print(tap, t, cycles(addrs), res)
